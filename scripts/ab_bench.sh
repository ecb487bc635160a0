#!/bin/bash
# Side-by-side bench.py lines of library builds on ONE box (scan_device path,
# ABI-stable across builds): ab_bench.sh TAG "bench args" lib1 lib2 ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out; TAG=$1; ARGS=$2; shift 2; mkdir -p "$OUT"
: > "$OUT/abb_$TAG.txt"
for pass in 1 2 3; do
  for lib in "$@"; do
    for mode in ${AB_MODES:-dense dense16 count}; do
      PM_LIBPM=$(pwd)/$lib timeout -k 10 300 python bench.py --no-cpu --steps 10 --mode $mode $ARGS > "$OUT/abb_tmp.json" 2>"$OUT/abb_err.txt" || { echo fail $lib; tail -5 "$OUT/abb_err.txt"; exit 1; }
      python3 -c "
import json; d=json.load(open('$OUT/abb_tmp.json'))
print('$pass', '$lib', '$mode', d['kernel_ms'], d['value'])" | tee -a "$OUT/abb_$TAG.txt"
    done
  done
done
