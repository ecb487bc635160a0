#!/bin/bash
# Counters of sparse-DFA variants on the lines stream (snort, 1 GiB, dense
# u32): SQ instruction / wait counters, TA / TD busy, L2 requests, hits and
# misses, fabric bytes; one rocprofv3 --pmc pass per group and variant.  Usage: gpu_pmc_sdfa_ab.sh TAG "VARIANTS"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/pmc_ab_${1:-x}; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for v in ${2:-12 24}; do
  i=0
  for grp in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
             "TA_TA_BUSY_sum TA_BUFFER_WAVEFRONTS_sum" "TD_TD_BUSY_sum" "TCP_TCC_WRITE_REQ_sum TCP_TCC_READ_REQ_sum" \
             "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1)); mkdir -p "$OUT/v$v"
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$OUT/v$v/p$i" -o c -- \
       python3 "$ROOT/scripts/sdfa_lds_ab.py" --streams lines --modes dense --variants $v --rounds 1 --nocheck 22,23,24,29,30,31 \
       > "$OUT/v$v/p$i.log" 2>&1 || { tail "$OUT/v$v/p$i.log"; exit 1; }
  done
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections, json, os
res = {}
for vd in sorted(glob.glob(sys.argv[1] + "/v*/")):
    agg = collections.defaultdict(list)
    for f in glob.glob(vd + "p*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "dfa_sparse" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    res[os.path.basename(vd.rstrip("/"))] = {c: sorted(v)[len(v) // 2] for c, v in agg.items()}
print(json.dumps(res, indent=1))
json.dump(res, open(sys.argv[1] + "/summary.json", "w"), indent=1)
PY
