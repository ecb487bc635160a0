#!/bin/bash
# Side-by-side timing of library builds on ONE box (box-to-box spread is
# larger than most single changes): ab_libs.sh TAG "SPARSE_AB_ARGS" lib1 lib2 ...
# Each build in its own process (PM_LIBPM), alternating, 3 passes, through
# scripts/sparse_ab.py; lines go to gpurun_out/ab_TAG.jsonl.  A lib named
# "libpm.so" is the in-tree product build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; TAG=$1; ARGS=$2; shift 2; mkdir -p "$OUT"
: > "$OUT/ab_$TAG.jsonl"
for pass in 1 2 3; do
  for lib in "$@"; do
    L=$ROOT/$lib; [ "$lib" = libpm.so ] && L=$ROOT/patternmatching_amd/libpm.so
    PM_LIBPM=$L timeout -k 10 300 python scripts/sparse_ab.py $ARGS > "$OUT/ab_${TAG}_tmp.json" 2> "$OUT/ab_${TAG}_tmp.err" \
        || { tail "$OUT/ab_${TAG}_tmp.err"; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$OUT/ab_${TAG}_tmp.json')); d['pass']=$pass; d['build']='$lib'; print(json.dumps(d))" \
        | tee -a "$OUT/ab_$TAG.jsonl" | cut -c1-400
  done
done
