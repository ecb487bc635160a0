#!/bin/bash
# SQ counters of the RT kernel's count-only launches, spill regions resolved
# at 16 chunks (the old default) and at 4 (the round-6 default), snort ASCII
# 1 GiB, one process per (cap, pass) (scripts/rt_spillcap_ab.py, --kernel-trace
# only), summarised per cap.  Usage: gpu_pmc_count.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/pmc_count_$1; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
PASSES=("SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
        "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum")
for cap in 16 4; do
  i=0
  for C in "${PASSES[@]}"; do
    i=$((i + 1))
    timeout -k 10 -s KILL 180 rocprofv3 --kernel-trace --pmc $C --output-format csv -d "$OUT/cap$cap/raw$i" -o c -- \
        python3 "$ROOT/scripts/rt_spillcap_ab.py" --streams ascii --modes count --caps $cap --rounds 2 > "$OUT/cap${cap}_pass$i.log" 2>&1 \
        || { tail "$OUT/cap${cap}_pass$i.log"; exit 1; }
  done
done
python3 - "$OUT" <<'PY'
import csv, glob, json, sys, statistics
res = {}
for cap in ("16", "4"):
    d = {}
    for f in glob.glob(f"{sys.argv[1]}/cap{cap}/raw*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "rt_scan_kernel" in r["Kernel_Name"]:
                d.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    res["cap" + cap] = {c: statistics.median(v) for c, v in d.items()}
    m = res["cap" + cap]
    if m.get("SQ_INSTS_LDS"):
        m["lds_conflict_cycles_per_lds_instr"] = m.get("SQ_LDS_BANK_CONFLICT", 0) / m["SQ_INSTS_LDS"]
    if m.get("SQ_WAVE_CYCLES"):
        m["wait_frac"] = m.get("SQ_WAIT_ANY", 0) / m["SQ_WAVE_CYCLES"]
json.dump(res, open(sys.argv[1] + "/summary.json", "w"), indent=1)
for k, d in res.items():
    print(k, {c: round(v / 1e6, 3) if v > 1000 else round(v, 3) for c, v in sorted(d.items())})
PY
