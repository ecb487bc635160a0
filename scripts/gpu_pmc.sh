#!/bin/bash
# PMC counters per kernel for the ablation variants (separate rocprofv3 passes,
# --pmc only with --kernel-trace).  Usage: gpu_pmc.sh TAG VARIANTS [mode]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; TAG=${1:-pmc}; mkdir -p "$OUT/pmc_$TAG"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$OUT/pmc_$TAG/p$i" -o c -- \
     python3 "$ROOT/scripts/bench_variants.py" --variants ${2:-0} --rounds 1 ${@:3} > "$OUT/pmc_$TAG/p$i.log" 2>&1 || { tail "$OUT/pmc_$TAG/p$i.log"; exit 1; }
done
python3 - "$OUT/pmc_$TAG" <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        name = name[:name.index("(", name.index("::") if "::" in name else 0)] if "(" in name else name
        agg[name.replace("(anonymous namespace)::", "")[-48:]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for kern, cs in agg.items():
    print("==", kern)
    for c, v in sorted(cs.items()):
        print(f"   {c:22s} median={sorted(v)[len(v)//2]:.4g} n={len(v)}")
PY
