#!/bin/bash
# HBM traffic of the bench workload's scan kernel from PMC counters, one
# counter per rocprofv3 pass (--pmc with --kernel-trace only).
# Usage: gpu_traffic.sh TAG [bench args...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; TAG=${1:-t}; mkdir -p "$OUT/traffic_$TAG"
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum; do
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d "$OUT/traffic_$TAG/$c" -o c -- \
    python3 "$ROOT/bench.py" --no-cpu --steps 3 --warmup 1 ${@:2} > "$OUT/traffic_$TAG/$c.log" 2>&1 || { tail "$OUT/traffic_$TAG/$c.log"; exit 1; }
done
python3 - "$OUT/traffic_$TAG" <<'PY'
import csv, glob, json, sys, statistics
res = {}
for f in glob.glob(sys.argv[1] + "/*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "scan_kernel" not in r["Kernel_Name"]:
            continue
        res.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
out = {k: statistics.median(v) for k, v in res.items()}
print(json.dumps(out, indent=1))
json.dump(out, open(sys.argv[1] + "/summary.json", "w"), indent=1)
PY
