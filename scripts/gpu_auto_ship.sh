#!/bin/bash
# The auto and ac kinds on the shipped stream (ids and count only) plus the
# DFA-form GPU tests; each GPU step has its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-auto_ship}; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread -k "forms or variants or fuzz or dfa or auto" > "$OUT/pytest_gpu.log" 2>&1 || { tail "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
for k in auto ac; do for m in dense count; do
  timeout -k 10 300 python -u bench.py --no-cpu --no-extra --stream ship --kernel $k --mode $m --steps 10 > "$OUT/ship_${k}_$m.json" 2> "$OUT/ship_${k}_$m.err" || { tail "$OUT/ship_${k}_$m.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/ship_${k}_$m.json')); print('ship', '$k', '$m', d['kernel_ms'], d['value'], d.get('last_kernel'))"
done; done
