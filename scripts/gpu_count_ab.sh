#!/bin/bash
# Count-only RT kernel: the product against its ablations (13: candidates
# dropped after classification, 14: pushed but no tail), side by side on one
# box, snort 1 GiB ASCII / lines / shipped.  Usage: gpu_count_ab.sh TAG [VARIANTS]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-count}; mkdir -p "$OUT"
for st in 0 3 2; do
  timeout -k 10 300 python scripts/bench_variants.py --variants ${2:-0,13,14} --modes count --rounds 5 --stream $st --counts \
      > "$OUT/count_stream$st.json" 2> "$OUT/count_stream$st.err" || { tail "$OUT/count_stream$st.err"; exit 1; }
  python3 -c "import json; d=json.load(open(\"$OUT/count_stream$st.json\")); print(\"stream $st\", {k: (v[\"ms\"] if isinstance(v, dict) else v) for k, v in d.items()})"
done
