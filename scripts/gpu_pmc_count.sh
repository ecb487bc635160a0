#!/bin/bash
# Instruction and LDS counters of the count-only RT kernel (1 GiB snort
# ASCII): the product (variant 0) and the chunk loop without the deep walks
# (variant 6), one rocprofv3 --pmc pass each (--kernel-trace only).
# Usage: gpu_pmc_count.sh TAG [VARIANTS]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/pmc_count_${1:-x}; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for v in ${2:-0 6}; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT \
      SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY --output-format csv -d "$OUT/v$v" -o c -- \
      python3 "$ROOT/scripts/bench_variants.py" --variants $v --modes count --rounds 1 > "$OUT/v$v.log" 2>&1 \
      || { tail "$OUT/v$v.log"; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections, json, os
res = {}
for vd in sorted(glob.glob(sys.argv[1] + "/v*/")):
    agg = collections.defaultdict(list)
    for f in glob.glob(vd + "**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "rt_scan" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    res[os.path.basename(vd.rstrip("/"))] = {c: sorted(v)[len(v) // 2] for c, v in agg.items()}
print(json.dumps(res, indent=1))
json.dump(res, open(sys.argv[1] + "/summary.json", "w"), indent=1)
PY
