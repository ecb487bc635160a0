#!/bin/bash
# rocprofv3 kernel stats of the ablation variants.  Usage: gpu_prof_variants.sh TAG VARIANTS [extra args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; TAG=${1:-p}; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/profv_$TAG" -o v -- \
  python3 "$ROOT/scripts/bench_variants.py" --variants ${2:-0} --rounds 3 ${@:3} > "$OUT/profv_$TAG.log" 2>&1 || { tail "$OUT/profv_$TAG.log"; exit 1; }
f=$(find "$OUT/profv_$TAG" -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f"{r['Name'][:70]:70s} calls={r['Calls']:>4} avg_us={float(r['AverageNs'])/1e3:9.1f} min_us={float(r['MinNs'])/1e3:9.1f}")
PY
