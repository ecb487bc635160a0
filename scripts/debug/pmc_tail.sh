#!/bin/bash
# PMC passes (one counter group per run) of RT variants 0 and 6 on the shipped stream
set -o pipefail
OUT=gpurun_out/pmc_tail; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for v in 0 6; do
 for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
  tag=$(echo $grp | cut -d' ' -f1)
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $R/$OUT/v${v}_$tag -o c -- python3 $R/scripts/debug/run_variant.py $v count ship 2 > $R/$OUT/v${v}_$tag.log 2>&1 || { tail -5 $R/$OUT/v${v}_$tag.log; exit 1; }
 done
done
python3 - $R/$OUT <<'PY'
import csv, glob, sys, collections
res = collections.defaultdict(dict)
for f in glob.glob(sys.argv[1] + "/*/**/*counter_collection.csv", recursive=True):
    v = f.split("/pmc_tail/")[1].split("_")[0]
    for r in csv.DictReader(open(f)):
        if "rt_scan_kernel" in r["Kernel_Name"]:
            res[v].setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
for v in sorted(res):
    print(v, {k: "%.4g" % (sum(x) / len(x)) for k, x in sorted(res[v].items())})
PY
