#!/bin/bash
# Round-4 session c: whole-line id stores through LDS (sparse DFA variants
# 19-21) against the product (12) and its LDS-less form (10), with the GPU
# tests that cover them; then instruction counters of the decoupled-lane
# kernel (13) beside the product (12) on the lines stream.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); TAG=${1:-r04c}; OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"
bash scripts/gpu_dyn.sh $TAG 12,10,19,20,21 lines,ship,ascii || exit 1
cd /tmp && export TMPDIR=/tmp
for v in 12 13; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS \
      SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY --output-format csv -d "$OUT/pmc_v$v" -o c -- \
      python3 "$ROOT/scripts/sdfa_lds_ab.py" --streams lines --modes dense --variants $v --rounds 1 \
      > "$OUT/pmc_v$v.log" 2>&1 || { tail "$OUT/pmc_v$v.log"; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections, json, os
res = {}
for vd in sorted(glob.glob(sys.argv[1] + "/pmc_v*/")):
    agg = collections.defaultdict(list)
    for f in glob.glob(vd + "**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "dfa_sparse" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    res[os.path.basename(vd.rstrip("/"))] = {c: sorted(v)[len(v) // 2] for c, v in agg.items()}
print(json.dumps(res, indent=1))
json.dump(res, open(sys.argv[1] + "/pmc_summary.json", "w"), indent=1)
PY
