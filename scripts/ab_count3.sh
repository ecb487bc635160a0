# A/B of the count-only chunk loop (cnt_perm: v_perm keys + two-bit class
# field, against cnt_old: the class sum) and of the all-loads-first LDS
# staging (stage = cnt_perm + staging): random ASCII / shipped / lines count,
# 1 GiB dense ASCII, et 64 MiB (C2) and 16 MiB dense; then the count and
# fuzz parity tests on the working tree
set -o pipefail
cd $GRAFT_REPO_ROOT
L="ablibs/cnt_old/libpm.so ablibs/cnt_perm/libpm.so ablibs/stage/libpm.so"
for st in 0 2 3; do AB_ARGS="--stream $st --modes count" bash scripts/ab_time.sh count3_s$st $L || exit 1; done
AB_ARGS="--modes dense,dense16" bash scripts/ab_time.sh stage_1g $L || exit 1
AB_ARGS="--dict et --bytes 67108864 --modes dense,count --rounds 20" bash scripts/ab_time.sh stage_c2 $L || exit 1
AB_ARGS="--dict et --bytes 16777216 --modes dense --rounds 20" bash scripts/ab_time.sh stage_16m $L || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_fuzz.py -k "count or fuzz or golden or digests" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_count3.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_count3.log; exit $rc
