#!/bin/bash
# Sparse DFA warm-up rule A/B (sync 0: max_len-1 bytes back; 1: from the last
# synchronizing 3-gram), ids (form 12) and count only (form 10), three streams;
# then the GPU suite on the same tree.  Each GPU step has its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-sync_ab}; mkdir -p "$OUT"
timeout -k 10 300 python -u scripts/sdfa_mlp_sweep.py --forms 12 --lanes 1024 --sync 0,1 --streams lines,ship,ascii --width 4 > "$OUT/ids.log" 2>&1 || { tail "$OUT/ids.log"; exit 1; }
tail -1 "$OUT/ids.log"
timeout -k 10 300 python -u scripts/sdfa_mlp_sweep.py --forms 12 --lanes 1024 --sync 0,1 --streams lines,ship --width 2 > "$OUT/u16.log" 2>&1 || { tail "$OUT/u16.log"; exit 1; }
tail -1 "$OUT/u16.log"
timeout -k 10 300 python -u scripts/sdfa_mlp_sweep.py --forms 10 --lanes 1024 --sync 0,1 --streams lines,ship,ascii --width 0 > "$OUT/count.log" 2>&1 || { tail "$OUT/count.log"; exit 1; }
tail -1 "$OUT/count.log"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -2 "$OUT/pytest_gpu.log"; exit $rc
