#!/bin/bash
# Dense coded rows, ids (u32 / u16): lanes per CU after the 3-gram warm-ups.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-dense_lanes}; mkdir -p "$OUT"
for w in 4 2; do
  timeout -k 10 300 python -u scripts/sdfa_mlp_sweep.py --sparse 0 --forms 12 --lanes 512,768,1024 --sync 1 --rounds 6 --streams ship,ascii --width $w > "$OUT/dense_w$w.log" 2>&1 || { tail "$OUT/dense_w$w.log"; exit 1; }
done
grep -h "ms$" "$OUT"/*.log
