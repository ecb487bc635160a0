set -o pipefail
OUT=gpurun_out/r02a; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -rf --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python __graft_entry__.py smoke > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
cat $OUT/bench.json
timeout -k 10 300 python bench.py --stream ship --no-cpu --steps 5 > $OUT/bench_ship.json 2>>$OUT/bench.err || exit $?
timeout -k 10 300 python bench.py --stream ship --kernel ac --no-cpu --steps 5 > $OUT/bench_ship_ac.json 2>>$OUT/bench.err || exit $?
cat $OUT/bench_ship.json $OUT/bench_ship_ac.json | cut -c1-300
