#!/bin/bash
# RT grid rule A/B: ablibs/base (one workgroup per CU) vs ablibs/grid (the
# size rule in rt_blocks), et and snort, 1 MiB .. 1 GiB, alternating passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out/grid; mkdir -p "$OUT"; : > "$OUT/ab.txt"
for pass in 1 2; do
for dict in et snort; do
for b in 1048576 4194304 16777216 33554432 67108864 1073741824; do
for lib in base grid; do
  PM_LIBPM=$(pwd)/ablibs/$lib/libpm.so timeout -k 10 120 python scripts/bench_variants.py --dict $dict --bytes $b \
      --variants 0 --rounds 7 > "$OUT/tmp.json" 2>&1 || { tail "$OUT/tmp.json"; exit 1; }
  grep -v amdgpu "$OUT/tmp.json" | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print('$pass $dict $b $lib', ' '.join(f\"{k.split('-')[1]}={v['ms']}\" for k,v in d.items()))" | tee -a "$OUT/ab.txt"
done; done; done; done
