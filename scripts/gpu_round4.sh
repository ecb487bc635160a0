#!/bin/bash
# Round-4 measurement session: GPU tests, smoke, the default bench line, the
# rocprofv3 kernel stats of the default bench (headline kernel, count-only,
# the deep leg) and the PMC traffic of the headline kernel.
# Usage: gpu_round4.sh TAG.  Every GPU step has its own time limit; the first
# failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); TAG=${1:-r04}; OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"
export PM_EVIDENCE_DIR=$OUT
echo "== $(date) host cpus $(nproc) share ${OMP_NUM_THREADS:-?}"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rf --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -2 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python __graft_entry__.py smoke > "$OUT/smoke.log" 2>&1 || { tail "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail "$OUT/bench.err"; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print('C3', d['value'], 'kernel_ms', d['kernel_ms'], 'frac', d['roofline']['frac'], 'count', d['count_only']['kernel_ms'], 'deep', d['deep']['kernel_ms'], d['deep']['picked'], 'cpu', d['cpu_baseline']['value'], d['cpu_baseline']['cores']); print({k: (v['kernel_ms'], v['stream_gbps'], v['roofline']['frac']) for k, v in d.get('configs', {}).items()})"
cd /tmp && export TMPDIR=/tmp
# kernel stats per leg, each its own run so a kernel's average is that leg's
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench -- \
    python3 "$ROOT/bench.py" --no-cpu --no-extra --steps 10 > "$OUT/bench_prof.json" 2> "$OUT/bench_prof.err" || { tail "$OUT/bench_prof.err"; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_count" -o bench -- \
    python3 "$ROOT/bench.py" --no-cpu --no-extra --mode count --steps 10 > "$OUT/bench_prof_count.json" 2> "$OUT/bench_prof_count.err" || { tail "$OUT/bench_prof_count.err"; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_deep" -o bench -- \
    python3 "$ROOT/bench.py" --no-cpu --no-extra --stream lines --kernel auto --steps 5 > "$OUT/bench_prof_deep.json" 2> "$OUT/bench_prof_deep.err" || { tail "$OUT/bench_prof_deep.err"; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d "$OUT/pmc/$c" -o c -- \
    python3 "$ROOT/bench.py" --no-cpu --no-extra --steps 3 --warmup 1 > "$OUT/pmc_$c.log" 2>&1 || { tail "$OUT/pmc_$c.log"; exit 1; }
done
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d "$OUT/pmc_deep/$c" -o c -- \
    python3 "$ROOT/bench.py" --no-cpu --no-extra --stream lines --kernel auto --steps 3 --warmup 1 > "$OUT/pmc_deep_$c.log" 2>&1 || { tail "$OUT/pmc_deep_$c.log"; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, statistics, json
for sub, pat, name in (("pmc", "rt_scan_kernel<0, 4", "pmc_summary.json"), ("pmc_deep", "dfa_sparse_stage", "pmc_deep_summary.json")):
    res = {}
    for f in glob.glob(sys.argv[1] + f"/{sub}/*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if pat in r["Kernel_Name"]:
                res.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    out = {k: statistics.median(v) for k, v in res.items()}
    json.dump(out, open(sys.argv[1] + "/" + name, "w"), indent=1)
    print(sub, out)
for leg in ("prof", "prof_count", "prof_deep"):
    for f in glob.glob(sys.argv[1] + f"/{leg}/**/*kernel_stats.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "rt_scan" in r["Name"] or "dfa_" in r["Name"]:
                print(leg, r["Name"][:60], "calls", r["Calls"], "avg_ns", r["AverageNs"])
PY
