#!/bin/bash
# Round-4 session b: the decoupled-lane DFA kernels against the product
# kernel (gpu_dyn.sh), the text-load shape probe (bw_probe5), the read_block
# host path at 100 KiB calls with and without zero copy (host_profile.py),
# and the count-only kernel's instruction counters (gpu_pmc_count.sh).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r04b}; mkdir -p "$OUT"
bash scripts/gpu_dyn.sh ${1:-r04b} || exit 1
timeout -k 10 120 ./scripts/bw_probe5 > "$OUT/bw_probe5.txt" || exit 1
cat "$OUT/bw_probe5.txt"
for zc in 0 1 3; do
  PM_HOST_ZC=$zc timeout -k 10 300 python scripts/host_profile.py > "$OUT/host_profile_zc$zc.json" 2> "$OUT/host_profile_zc$zc.err" || { tail "$OUT/host_profile_zc$zc.err"; exit 1; }
  cat "$OUT/host_profile_zc$zc.json"
done
bash scripts/gpu_pmc_count.sh ${1:-r04b}
