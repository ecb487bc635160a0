#!/bin/bash
# Lanes per CU after the 3-gram warm-ups (shorter segments cost less now):
# sparse ids / count only and dense rows, 1 GiB snort.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-sync_lanes}; mkdir -p "$OUT"
timeout -k 10 300 python -u scripts/sdfa_mlp_sweep.py --forms 12 --lanes 512,1024,1536,2048 --sync 1 --streams lines,ship --width 4 > "$OUT/sparse_ids.log" 2>&1 || { tail "$OUT/sparse_ids.log"; exit 1; }
timeout -k 10 300 python -u scripts/sdfa_mlp_sweep.py --forms 10 --lanes 512,1024,1536,2048 --sync 1 --streams lines,ship --width 0 > "$OUT/sparse_count.log" 2>&1 || { tail "$OUT/sparse_count.log"; exit 1; }
timeout -k 10 300 python -u scripts/sdfa_mlp_sweep.py --sparse 0 --forms 12 --lanes 256,512,1024,2048 --sync 1 --streams ship,ascii --width 4 > "$OUT/dense_ids.log" 2>&1 || { tail "$OUT/dense_ids.log"; exit 1; }
timeout -k 10 300 python -u scripts/sdfa_mlp_sweep.py --sparse 0 --forms 12 --lanes 256,512,1024,2048 --sync 1 --streams ship,ascii --width 0 > "$OUT/dense_count.log" 2>&1 || { tail "$OUT/dense_count.log"; exit 1; }
grep -h "ms$" "$OUT"/*.log
