#!/bin/bash
# Quick GPU session: parity suite, smoke, the default bench line and the
# adversarial-stream lines.  Usage: g_quick.sh TAG [extra bench runs...]
set -o pipefail
OUT=gpurun_out/${1:-quick}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -rf --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python __graft_entry__.py smoke > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
run() {  # name, bench args
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > "$OUT/bench_$name.json" 2> "$OUT/bench_$name.err" || { tail "$OUT/bench_$name.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$name.json')); print('$name', d['value'], d['unit'], 'kernel_ms', d['kernel_ms'], 'frac', d['roofline']['frac'], d.get('accuracy', ''))"
}
run dense --no-cpu
run dense16 --mode dense16 --no-cpu
run count --mode count --no-cpu
run ship --stream ship --no-cpu --steps 5
run ship_score --stream ship --no-cpu --steps 3 --score
run ship_ac --stream ship --kernel ac --no-cpu --steps 5
