#!/bin/bash
# Parity tests + ablation timings (no profiler).  Usage: gpu_quick.sh TAG [variants]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out; TAG=${1:-q}; mkdir -p "$OUT"
timeout -k 10 900 python -m pytest tests -m gpu -q -x -rf ${PYTEST_ARGS:-} > "$OUT/pytest_gpu_$TAG.log" 2>&1
rc=$?; tail -4 "$OUT/pytest_gpu_$TAG.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_variants.py --variants ${2:-0,1,2,3} > "$OUT/variants_$TAG.json" 2>&1 || { tail "$OUT/variants_$TAG.json"; exit 1; }
grep -v amdgpu.ids "$OUT/variants_$TAG.json" | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
for k,v in d.items(): print(k, {a: round(b, 1) for a, b in v.items()}) if 'ms' not in v else print(k, v['ms'], 'stream GB/s', v['GBps_stream'], 'alg GB/s', v['alg_GBps'])"
