#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
TAG=${1:-r01}
mkdir -p "$OUT"
echo "== host: $(nproc) cpus; $(date)"
rocm-smi --showproductname 2>/dev/null | grep -i "card series" | head -2
timeout -k 10 900 python -m pytest tests -m gpu -q -rf ${PYTEST_ARGS:-} > "$OUT/pytest_gpu_$TAG.log" 2>&1
rc=$?; tail -5 "$OUT/pytest_gpu_$TAG.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python __graft_entry__.py smoke > "$OUT/smoke_$TAG.log" 2>&1 || exit $?
cat "$OUT/smoke_$TAG.log"
timeout -k 10 600 python bench.py > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err" || { tail "$OUT/bench_$TAG.err"; exit 1; }
cat "$OUT/bench_$TAG.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o bench -- \
    python3 "$ROOT/bench.py" --no-cpu --steps 10 > "$OUT/bench_prof_$TAG.json" 2> "$OUT/bench_prof_$TAG.err" || { tail "$OUT/bench_prof_$TAG.err"; exit 1; }
cat "$OUT/bench_prof_$TAG.json"
find "$OUT/prof_$TAG" -name "*stats*" | head
