#!/bin/bash
# Count-only RT kernel, library builds side by side on one box (alternating,
# 3 passes, scripts/rt_spillcap_ab.py): ab_count.sh TAG lib1 lib2 ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; TAG=$1; shift; mkdir -p "$OUT"
: > "$OUT/ab_$TAG.jsonl"
for pass in 1 2 3; do
  for lib in "$@"; do
    L=$ROOT/$lib; [ "$lib" = libpm.so ] && L=$ROOT/patternmatching_amd/libpm.so
    PM_LIBPM=$L timeout -k 10 300 python scripts/rt_spillcap_ab.py --streams ascii,ship,lines --modes count --caps 0 --rounds 5 \
        > "$OUT/ab_${TAG}_tmp.json" 2> "$OUT/ab_${TAG}_tmp.err" || { tail "$OUT/ab_${TAG}_tmp.err"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/ab_${TAG}_tmp.json')); d['pass']=$pass; d['build']='$lib'; print(json.dumps(d))" \
        | tee -a "$OUT/ab_$TAG.jsonl" | cut -c1-300
  done
done
