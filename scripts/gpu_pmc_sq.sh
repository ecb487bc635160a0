#!/bin/bash
# SQ counters (one rocprofv3 --pmc pass, --kernel-trace only) of a bench
# workload's kernels: the headline run also launches the RT kernel's
# streaming floor (rt_scan_kernel<2, 4>) after its timed steps, so one pass
# gives the product kernel and its floor side by side.
# Usage: gpu_pmc_sq.sh TAG [bench args...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/pmc_sq_$1; mkdir -p "$OUT"
shift
cd /tmp && export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
timeout -k 10 120 rocprofv3 --kernel-trace --pmc $C --output-format csv -d "$OUT/raw" -o c -- \
    python3 "$ROOT/bench.py" --no-cpu --no-extra --steps 3 --warmup 1 "$@" > "$OUT/bench.log" 2>&1 \
    || { tail "$OUT/bench.log"; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, json, sys, statistics
res = {}
for f in glob.glob(sys.argv[1] + "/raw/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "rt_scan" in k or "dfa_" in k:
            res.setdefault(k, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
out = {k: {c: statistics.median(v) for c, v in d.items()} for k, d in res.items()}
json.dump(out, open(sys.argv[1] + "/summary.json", "w"), indent=1)
for k, d in out.items():
    lds = d.get("SQ_INSTS_LDS", 0) or 1
    print(k[:60], {c: round(v / 1e6, 2) for c, v in d.items()}, "conflict cycles per LDS instr",
          round(d.get("SQ_LDS_BANK_CONFLICT", 0) / lds, 2))
PY
