#!/bin/bash
# Side-by-side bench.py legs of library builds on ONE box:
#   bench_ab.sh TAG "BENCH_ARGS" lib1 lib2 ...
# Each build in its own process (PM_LIBPM), alternating, 3 passes; one JSON
# line per run ({"build", "pass", "kernel_ms", "value"}) to
# gpurun_out/bab_TAG.jsonl.  A lib named "libpm.so" is the in-tree build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; TAG=$1; ARGS=$2; shift 2; mkdir -p "$OUT"
: > "$OUT/bab_$TAG.jsonl"
for pass in 1 2 3; do
  for lib in "$@"; do
    L=$ROOT/$lib; [ "$lib" = libpm.so ] && L=$ROOT/patternmatching_amd/libpm.so
    PM_LIBPM=$L timeout -k 10 300 python bench.py --no-cpu --no-extra $ARGS > "$OUT/bab_${TAG}_tmp.json" 2> "$OUT/bab_${TAG}_tmp.err" \
        || { tail "$OUT/bab_${TAG}_tmp.err"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/bab_${TAG}_tmp.json')); print(json.dumps({'build': '$lib', 'pass': $pass, 'args': '$ARGS', 'kernel_ms': d['kernel_ms'], 'value': d['value']}))" \
        | tee -a "$OUT/bab_$TAG.jsonl"
  done
done
