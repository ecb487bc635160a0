#!/bin/bash
# Quick GPU check: a pytest selection (-k EXPR) and optional bench commands,
# each under its own time limit; the first failure ends the script.
# Usage: gpu_quick.sh TAG 'PYTEST_K' ['BENCH ARGS' ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; K=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export PM_EVIDENCE_DIR=$OUT
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rf --timeout 300 --timeout-method thread -k "$K" > "$OUT/pytest.log" 2>&1
  rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
fi
i=0
for a in "$@"; do
  i=$((i+1))
  timeout -k 10 600 python bench.py --no-cpu $a > "$OUT/bench_$i.json" 2> "$OUT/bench_$i.err" || { tail "$OUT/bench_$i.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/bench_$i.json')); print('$a', '->', d['kernel_ms'], 'ms', d['value'], 'GB/s', d['config']['kernel'][-60:])"
done
