#!/bin/bash
# GPU session for the AC-DFA forms: the GPU suite, then bench lines of the
# ac / auto kinds on the three streams and a sparse-form shape sweep.
# Usage: gpu_dfa_forms.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-forms}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -rf --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
run() {  # name, bench args
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > "$OUT/bench_$name.json" 2> "$OUT/bench_$name.err" || { tail "$OUT/bench_$name.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$name.json')); print('$name', d['value'], d['unit'], 'kernel_ms', d['kernel_ms'], d['config']['kernel'])"
}
for st in ship lines ascii; do
  run ${st}_ac --stream $st --kernel ac --no-cpu --steps 5
  run ${st}_auto --stream $st --kernel auto --no-cpu --steps 5
done
run lines_rt --stream lines --no-cpu --steps 5
timeout -k 10 300 python scripts/dfa_coded_sweep.py --forms 1 --lanes ${SWEEP_LANES:-384,512,768} --chains 1 --blocks 16,32 > $OUT/sweep.txt 2>&1 || exit $?
grep -v amdgpu $OUT/sweep.txt | grep -v "^{"
