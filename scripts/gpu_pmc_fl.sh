#!/bin/bash
# Deep-kernel PMC before/after: the round-4 product sparse kernel
# (sparse_kernel 2, u16-staged 8-B units) and the round-5 fallback-linked one
# (sparse_kernel 1) on the same 1 GiB snort lines stream, one process per
# counter pass (scripts/sparse_ab.py, --kernel-trace only), summarised per
# kernel name.  Usage: gpu_pmc_fl.sh TAG [sparse_ab args...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/pmc_fl_$1; mkdir -p "$OUT"
shift
ARGS=${*:-"--dict snort --streams lines --kernels 1,2 --rounds 2"}
cd /tmp && export TMPDIR=/tmp
PASSES=("FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum"
        "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD")
i=0
for C in "${PASSES[@]}"; do
  i=$((i + 1))
  timeout -k 10 -s KILL 180 rocprofv3 --kernel-trace --pmc $C --output-format csv -d "$OUT/raw$i" -o c -- \
      python3 "$ROOT/scripts/sparse_ab.py" $ARGS > "$OUT/pass$i.log" 2>&1 \
      || { tail "$OUT/pass$i.log"; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, json, sys, statistics
res = {}
for f in glob.glob(sys.argv[1] + "/raw*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "dfa_" in k:
            k = k.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
            res.setdefault(k, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
out = {k: {c: statistics.median(v) for c, v in d.items()} for k, d in res.items()}
json.dump(out, open(sys.argv[1] + "/summary.json", "w"), indent=1)
for k, d in out.items():
    print(k[:70])
    print("  ", {c: round(v / 1e6, 2) for c, v in sorted(d.items())}, "(millions)")
PY
