#!/bin/bash
# Full measurement session on one GPU box: parity tests, smoke, every bench
# line of DESIGN.md §4 (BASELINE configs 2, 3 and 5 plus the u16 / count / AC
# modes), rocprofv3 kernel stats of the default bench and its PMC traffic.
# Usage: gpu_round.sh TAG.  Every GPU step has its own time limit; the first
# failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/round_${1:-r}; mkdir -p "$OUT"
echo "== $(date) host cpus $(nproc)"
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -rf --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python __graft_entry__.py smoke > "$OUT/smoke.log" 2>&1 || exit $?
tail -1 "$OUT/smoke.log"
run() {  # name, bench args
  local name=$1; shift
  timeout -k 10 900 python bench.py "$@" > "$OUT/bench_$name.json" 2> "$OUT/bench_$name.err" || { tail "$OUT/bench_$name.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/bench_$name.json')); print('$name', d['value'], d['unit'], 'kernel_ms', d['kernel_ms'], 'frac', d['roofline']['frac'])"
}
run dense
run dense16 --mode dense16 --no-cpu
run count --mode count --no-cpu
run ac --kernel ac --no-cpu --steps 5
run c2_et64m --dict et --bytes 67108864 --no-cpu
run c5_merged4g --dict merged --bytes 4294967296 --no-cpu --steps 10
run score --score --no-cpu --steps 5
run ship --stream ship --no-cpu --steps 5
run ship_count --stream ship --mode count --no-cpu --steps 5
run ship_ac --stream ship --kernel ac --no-cpu --steps 5
run ship_auto --stream ship --kernel auto --no-cpu --steps 5
run lines --stream lines --no-cpu --steps 5
run lines_ac --stream lines --kernel ac --no-cpu --steps 5
run lines_auto --stream lines --kernel auto --no-cpu --steps 5
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench -- \
    python3 "$ROOT/bench.py" --no-cpu --steps 10 > "$OUT/bench_prof.json" 2> "$OUT/bench_prof.err" || { tail "$OUT/bench_prof.err"; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_lines_ac" -o bench -- \
    python3 "$ROOT/bench.py" --no-cpu --steps 5 --stream lines --kernel ac > "$OUT/bench_prof_lines_ac.json" 2> "$OUT/bench_prof_lines_ac.err" || { tail "$OUT/bench_prof_lines_ac.err"; exit 1; }
for c in FETCH_SIZE WRITE_SIZE TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum; do
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d "$OUT/pmc/$c" -o c -- \
    python3 "$ROOT/bench.py" --no-cpu --steps 3 --warmup 1 > "$OUT/pmc_$c.log" 2>&1 || { tail "$OUT/pmc_$c.log"; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, json, sys, statistics
res = {}
for f in glob.glob(sys.argv[1] + "/pmc/*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "rt_scan_kernel<0, 4" in r["Kernel_Name"]:  # the product kernel (bench also runs the floor variant)
            res.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
out = {k: statistics.median(v) for k, v in res.items()}
print(json.dumps(out))
json.dump(out, open(sys.argv[1] + "/pmc_summary.json", "w"), indent=1)
for f in glob.glob(sys.argv[1] + "/prof/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "rt_scan_kernel<0, 4" in r["Name"]:
            print("rocprof", r["Name"][:60], "calls", r["Calls"], "avg_ns", r["AverageNs"])
PY
