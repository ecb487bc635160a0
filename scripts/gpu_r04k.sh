#!/bin/bash
# Round 4, late: gids ordered by pattern length (fewer escapes in the coded
# DFA words) -- the whole GPU suite, then the staged sparse kernel with 1 /
# 4 / 8 escapes per lane per round, side by side, ids checked equal.
# Usage: gpu_r04k.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r04k}; mkdir -p "$OUT"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 600 python scripts/sdfa_lds_ab.py --variants ${VARIANTS:-28,32,33} --rounds 5 \
    > "$OUT/escape_rounds_ab.json" 2> "$OUT/escape_rounds_ab.err" || { tail "$OUT/escape_rounds_ab.err"; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/escape_rounds_ab.json'))
for k,v in d.items(): print(k, v if not isinstance(v, dict) else v.get('ms', v))"
