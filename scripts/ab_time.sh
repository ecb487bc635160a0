#!/bin/bash
# Side-by-side timing of library builds on ONE box: ab_time.sh TAG lib1 lib2 ...
# (each build in its own process, alternating, 3 passes; box-to-box variance
# is larger than most single changes).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out; TAG=$1; shift; mkdir -p "$OUT"
: > "$OUT/ab_$TAG.txt"
for pass in 1 2 3; do
  for lib in "$@"; do
    PM_LIBPM=$(pwd)/$lib timeout -k 10 300 python scripts/bench_variants.py --variants 0 --rounds 5 ${AB_ARGS:-} \
        > "$OUT/ab_${TAG}_tmp.json" 2>&1 || { tail "$OUT/ab_${TAG}_tmp.json"; exit 1; }
    grep -v amdgpu "$OUT/ab_${TAG}_tmp.json" | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print('$pass', '$lib', ' '.join(f\"{k.split('-')[1]}={v['ms']}\" for k,v in d.items()))" | tee -a "$OUT/ab_$TAG.txt"
  done
done
