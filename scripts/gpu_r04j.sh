#!/bin/bash
# Round 4, late: the reference's loop with the batch call (GPU test), and the
# staged sparse kernel against its ablations (28 product; 29 no escape
# lookups, 30 no stores, 31 neither staging nor stores), side by side.
# Usage: gpu_r04j.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r04j}; mkdir -p "$OUT"
PM_EVIDENCE_DIR="$OUT" timeout -k 10 900 python -u -m pytest tests/test_integration.py -m gpu -x -v --timeout 850 \
    --timeout-method thread > "$OUT/pytest_integration.log" 2>&1 || { tail -30 "$OUT/pytest_integration.log"; exit 1; }
tail -3 "$OUT/pytest_integration.log"
timeout -k 10 600 python scripts/sdfa_lds_ab.py --variants 28,29,30,31 --nocheck 29,30,31 --rounds 5 \
    > "$OUT/stage_ablations.json" 2> "$OUT/stage_ablations.err" || { tail "$OUT/stage_ablations.err"; exit 1; }
cat "$OUT/stage_ablations.json" | python3 -c "
import json,sys; d=json.load(sys.stdin)
for k,v in d.items(): print(k, v if not isinstance(v, dict) else v.get('ms', v))"
