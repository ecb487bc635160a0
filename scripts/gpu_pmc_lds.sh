#!/bin/bash
# LDS / VALU pressure counters of rt_scan_kernel (one rocprofv3 --pmc pass per
# group).  Usage: gpu_pmc_lds.sh TAG VARIANTS MODES
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; TAG=${1:-lds}; mkdir -p "$OUT/pmc_$TAG"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES" \
           "SQ_WAVES SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$OUT/pmc_$TAG/p$i" -o c -- \
     python3 "$ROOT/scripts/bench_variants.py" --variants ${2:-0} --rounds 1 --modes ${3:-count} > "$OUT/pmc_$TAG/p$i.log" 2>&1 || { tail "$OUT/pmc_$TAG/p$i.log"; exit 1; }
done
python3 - "$OUT/pmc_$TAG" <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        if "rt_scan" not in name: continue
        key = name[name.index("rt_scan_kernel"):name.index("(", name.index("rt_scan_kernel"))]
        agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
for kern, cs in sorted(agg.items()):
    print("==", kern)
    for c, v in sorted(cs.items()):
        print(f"   {c:22s} median={sorted(v)[len(v)//2]:.4g} n={len(v)}")
PY
