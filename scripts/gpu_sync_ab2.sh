#!/bin/bash
# Warm-up rule A/B for the dense coded DFA (sync 0 / 1) and the sparse form
# again after the shared helper; the forms-agree and variants GPU tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-sync_ab2}; mkdir -p "$OUT"
timeout -k 10 300 python -u scripts/sdfa_mlp_sweep.py --sparse 0 --forms 12 --lanes 512 --sync 0,1 --streams lines,ship,ascii --width 4 > "$OUT/dense_ids.log" 2>&1 || { tail "$OUT/dense_ids.log"; exit 1; }
tail -1 "$OUT/dense_ids.log"
timeout -k 10 300 python -u scripts/sdfa_mlp_sweep.py --sparse 0 --forms 12 --lanes 512 --sync 0,1 --streams lines,ship --width 2 > "$OUT/dense_u16.log" 2>&1 || { tail "$OUT/dense_u16.log"; exit 1; }
tail -1 "$OUT/dense_u16.log"
timeout -k 10 300 python -u scripts/sdfa_mlp_sweep.py --sparse 0 --forms 10 --lanes 512 --sync 0,1 --streams lines,ship,ascii --width 0 > "$OUT/dense_count.log" 2>&1 || { tail "$OUT/dense_count.log"; exit 1; }
tail -1 "$OUT/dense_count.log"
timeout -k 10 300 python -u scripts/sdfa_mlp_sweep.py --forms 12 --lanes 1024 --sync 0,1 --streams lines,ship --width 4 > "$OUT/sparse_ids.log" 2>&1 || { tail "$OUT/sparse_ids.log"; exit 1; }
tail -1 "$OUT/sparse_ids.log"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread -k "forms or variants or fuzz or kmp or golden" > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -2 "$OUT/pytest_gpu.log"; exit $rc
