# the sparse-form kernel variants side by side, then the GPU parity suite
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/sdfa
timeout -k 10 600 python scripts/sdfa_lds_ab.py --modes dense,count --variants 0,1,2,3,4 > gpurun_out/sdfa/ab.json 2> gpurun_out/sdfa/ab.err || { tail gpurun_out/sdfa/ab.err; exit 1; }
cat gpurun_out/sdfa/ab.json
bash scripts/gpu_pmc_sdfa.sh a "0 1 2 3 4" > gpurun_out/sdfa/pmc.log 2>&1 || { tail gpurun_out/sdfa/pmc.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_fuzz.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/sdfa/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/sdfa/pytest.log; exit $rc
