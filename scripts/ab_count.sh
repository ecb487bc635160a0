# A/B of the count-only path (old u16 t12 vs the t8 byte table), then parity
set -o pipefail
cd $GRAFT_REPO_ROOT
for st in 0 2 3; do AB_ARGS="--stream $st --modes count,dense" bash scripts/ab_time.sh count_s$st ablibs/old/libpm.so ablibs/t8/libpm.so || exit 1; done
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_fuzz.py tests/test_bench.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_count.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_count.log; exit $rc
