#!/bin/bash
# read_block at the reference's 100 KiB chunks: the small RT kernel with its
# text window staged in LDS or read in place, and the spin wait, side by side
# (scripts/host_profile.py), after the parity tests that cover both forms.
# Usage: gpu_small_ab.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-small}; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "rt_small or read_block or ragged or edge or kmp or shards or small_gid or state_carries or pipeline" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
PM_HOST_VARIANTS=${VARIANTS:-stage0,stage1,stage1spin,stage0,stage1,stage1spin} PM_HOST_KINDS=${KINDS:-rt,ac} \
    timeout -k 10 300 python scripts/host_profile.py > "$OUT/host_profile.json" 2> "$OUT/host_profile.err" || { tail "$OUT/host_profile.err"; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/host_profile.json'))
for k, v in d.items():
    if isinstance(v, dict): print(k, v['GBps'], v['us_per_call'], 'wait', v['wait_us'], 'result', v['result_us'], 'dev', v['device_us'])"
