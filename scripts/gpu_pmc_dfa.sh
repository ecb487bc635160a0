#!/bin/bash
# PMC counters of the AC-DFA kernels, one rocprofv3 pass per counter group
# (--pmc with --kernel-trace only): bench.py --kernel ac on the shipped
# stream (holds the dense form) and the lines stream (holds the sparse
# form); per-kernel medians.  Usage: gpu_pmc_dfa.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/pmc_dfa_${1:-x}; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for st in ship lines; do
  i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES"; do
    i=$((i+1)); mkdir -p "$OUT/$st"
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$OUT/$st/p$i" -o c -- \
       python3 "$ROOT/bench.py" --stream $st --kernel ac --no-cpu --steps 2 --warmup 0 > "$OUT/$st/p$i.log" 2>&1 || { tail "$OUT/$st/p$i.log"; exit 1; }
  done
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections, json
res = {}
for st in ("ship", "lines"):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{sys.argv[1]}/{st}/p*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].replace("(anonymous namespace)::", "")
            name = name[:name.index("(")] if "(" in name else name
            if "dfa_" in name:
                agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res[st] = {k: {c: sorted(v)[len(v) // 2] for c, v in cs.items()} for k, cs in agg.items()}
print(json.dumps(res, indent=1))
json.dump(res, open(sys.argv[1] + "/summary.json", "w"), indent=1)
PY
