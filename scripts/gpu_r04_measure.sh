#!/bin/bash
# Round-4 measurement session on the tree as it stands:
#  1. PMC of the deep product kernel (dfa_sparse_lds_kernel, the sparse
#     AC-DFA form's variant 12) on the lines stream, snort, 1 GiB, dense u32
#     and count only: one rocprofv3 --pmc pass per counter group;
#  2. rocprofv3 --kernel-trace --stats of the other BASELINE configs on the
#     current kernels: C5 (merged, 4 GiB ASCII, rt, dense u32), C2 (et, 64
#     MiB, rt, dense u32) and merged x deep (the lines stream through auto).
# Usage: gpu_r04_measure.sh TAG [skip-pmc].  Each GPU step has its own limit;
# the first failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); TAG=${1:-r04a}; OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"
echo "== $(date) host cpus $(nproc) share ${OMP_NUM_THREADS:-?}"
cd /tmp && export TMPDIR=/tmp
if [ "${2:-}" != "skip-pmc" ]; then
  for mode in dense count; do
    i=0
    for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum" \
               "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY"; do
      i=$((i+1)); mkdir -p "$OUT/pmc_$mode"
      timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$OUT/pmc_$mode/p$i" -o c -- \
         python3 "$ROOT/scripts/sdfa_lds_ab.py" --streams lines --modes $mode --variants 12 --rounds 1 \
         > "$OUT/pmc_$mode/p$i.log" 2>&1 || { tail "$OUT/pmc_$mode/p$i.log"; exit 1; }
    done
  done
  python3 - "$OUT" <<'PY'
import csv, glob, sys, collections, json, os
res = {}
for md in sorted(glob.glob(sys.argv[1] + "/pmc_*")):
    agg = collections.defaultdict(list)
    for f in glob.glob(md + "/p*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "dfa_sparse" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    res[os.path.basename(md)] = {c: sorted(v)[len(v) // 2] for c, v in agg.items()}
print(json.dumps(res, indent=1))
json.dump(res, open(sys.argv[1] + "/deep_pmc_summary.json", "w"), indent=1)
PY
fi
run_prof() {  # name, limit, bench args...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$name" -o bench -- \
      python3 "$ROOT/bench.py" --no-cpu --no-extra "$@" > "$OUT/$name.json" 2> "$OUT/$name.err" \
      || { tail "$OUT/$name.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$name.json')); print('$name', d['value'], 'GB/s kernel_ms', d['kernel_ms'], 'frac', d['roofline']['frac'], d['config']['kernel'][:90])"
}
run_prof c5_merged_4g_rt 600 --dict merged --bytes 4294967296 --steps 10
run_prof c2_et_64m_rt 300 --dict et --bytes 67108864 --steps 20
run_prof merged_lines_auto 600 --dict merged --stream lines --kernel auto --steps 5
run_prof snort_lines_auto 600 --stream lines --kernel auto --steps 5
python3 - "$OUT" <<'PY'
import csv, glob, sys
for f in sorted(glob.glob(sys.argv[1] + "/prof_*/**/*kernel_stats.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        if "rt_scan" in r["Name"] or "dfa_" in r["Name"]:
            print(f.split("/prof_")[1].split("/")[0], r["Name"][:64], "calls", r["Calls"], "avg_ns", r["AverageNs"])
PY
