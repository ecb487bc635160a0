# A/B of count-only forms, then the count parity tests
set -o pipefail
cd $GRAFT_REPO_ROOT
for st in 0 3; do AB_ARGS="--stream $st --modes count" bash scripts/ab_time.sh count2_s$st ablibs/t8/libpm.so ablibs/t8sum/libpm.so || exit 1; done
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_fuzz.py -k "count or fuzz" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_count2.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_count2.log; exit $rc
