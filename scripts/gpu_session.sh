#!/bin/bash
# One GPU-box session: GPU tests, smoke, the default bench line.
# Usage: gpu_session.sh TAG [pytest selection...].  Every GPU step has its own
# time limit; the first failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); TAG=${1:-s}; shift; OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"
export PM_EVIDENCE_DIR=$OUT
echo "== $(date) host cpus $(nproc) share ${OMP_NUM_THREADS:-?}"
timeout -k 10 900 python -u -m pytest ${@:-tests} -m gpu -x -v -rf --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python __graft_entry__.py smoke > "$OUT/smoke.log" 2>&1 || { tail "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
