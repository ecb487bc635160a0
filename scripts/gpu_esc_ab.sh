#!/bin/bash
# The staged sparse kernel with 1 / 4 / 8 escapes per lane per round, side by
# side, ids checked equal (scripts/sdfa_lds_ab.py).  Usage: gpu_esc_ab.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-esc}; mkdir -p "$OUT"
timeout -k 10 600 python scripts/sdfa_lds_ab.py --variants ${VARIANTS:-28,32,33} --rounds 5 --modes ${MODES:-dense} \
    > "$OUT/escape_rounds_ab.json" 2> "$OUT/escape_rounds_ab.err" || { tail "$OUT/escape_rounds_ab.err"; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/escape_rounds_ab.json'))
for k,v in d.items(): print(k, v if not isinstance(v, dict) else v.get('ms', v))"
