#!/bin/bash
# L2 hit/miss and HBM request counters per RT variant (separate passes).
# Usage: gpu_pmc_l2.sh TAG VARIANTS MODES
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; TAG=${1:-l2}; mkdir -p "$OUT/pmc_$TAG"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" "TCC_EA0_RDREQ_32B_sum TCC_EA0_WRREQ_64B_sum" "TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$OUT/pmc_$TAG/p$i" -o c -- \
     python3 "$ROOT/scripts/bench_variants.py" --variants ${2:-0} --rounds 1 --modes ${3:-dense} > "$OUT/pmc_$TAG/p$i.log" 2>&1 || { tail "$OUT/pmc_$TAG/p$i.log"; exit 1; }
done
python3 - "$OUT/pmc_$TAG" <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        if "rt_scan" not in name: continue
        name = name[:name.index("(", name.index("::") if "::" in name else 0)] if "(" in name else name
        agg[name.replace("(anonymous namespace)::", "")[-40:]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for kern, cs in agg.items():
    print("==", kern)
    for c, v in sorted(cs.items()):
        print(f"   {c:24s} median={sorted(v)[len(v)//2]:.4g} n={len(v)}")
PY
