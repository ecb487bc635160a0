#!/bin/bash
# The sparse AC-DFA form's decoupled-lane kernels (pm_hip_debug_dfa_lds 13-18)
# against the round-3 product kernel (12), side by side on one box, ids and
# counts checked equal across variants (scripts/sdfa_lds_ab.py), then the
# GPU tests that cover them.  Usage: gpu_dyn.sh TAG [VARIANTS] [STREAMS]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); TAG=${1:-dyn}; OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"
V=${2:-12,13,14,15,16,17,18}
S=${3:-lines,ship,ascii}
timeout -k 10 400 python scripts/sdfa_lds_ab.py --streams $S --modes ${MODES:-dense,count} --variants $V --rounds 3 --nocheck ${NOCHECK:-none} \
    > "$OUT/ab.json" 2> "$OUT/ab.err" || { tail -20 "$OUT/ab.err"; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/ab.json'))
for k, v in d.items(): print(k, v['ms'], v['stream_gbps'])"
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
      -k "sparse_dfa_kernel_variants_agree or warmups_stop or first_scan_device or spill_cap_raised or graph_capture" \
      > "$OUT/pytest.log" 2>&1; rc=$?; tail -3 "$OUT/pytest.log"; exit $rc
fi
