#!/bin/bash
# Host-path (read_block from host memory) rates of library builds side by
# side on one box: host_ab.sh "chunk sizes" lib1 lib2 ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out; CHUNKS=$1; shift; mkdir -p "$OUT"
: > "$OUT/host_ab.txt"
for pass in 1 2; do
  for c in $CHUNKS; do
    for lib in "$@"; do
      PM_LIBPM=$(pwd)/$lib PM_HOST_CHUNK=$c PM_HOST_BYTES=$((c >= 1048576 ? 1073741824 : 268435456)) \
        timeout -k 10 300 python scripts/host_path_rate.py > "$OUT/host_tmp.json" 2> "$OUT/host_err.txt" || { echo fail $lib; tail -5 "$OUT/host_err.txt"; exit 1; }
      python3 -c "
import json; t=open('$OUT/host_tmp.json').read(); d=json.loads(t[t.index('{'):])
print('$pass', '$c', '$lib', {k: v for k, v in d.items() if k.endswith('GBps') and 'pcie' not in k})" | tee -a "$OUT/host_ab.txt"
    done
  done
done
