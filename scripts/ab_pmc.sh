#!/bin/bash
# HBM traffic (PMC FETCH_SIZE / WRITE_SIZE, one counter per pass) of the
# default bench line for library builds side by side: ab_pmc.sh lib1 lib2 ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/abpmc; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for lib in "$@"; do
  tag=$(basename "$lib" .so)
  for c in FETCH_SIZE WRITE_SIZE; do
    PM_LIBPM=$ROOT/$lib timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d "$OUT/$tag/$c" -o c -- \
      python3 "$ROOT/bench.py" --no-cpu --steps 3 --warmup 1 > "$OUT/${tag}_$c.log" 2>&1 || { tail "$OUT/${tag}_$c.log"; exit 1; }
  done
done
python3 - "$OUT" <<'PY'
import csv, glob, os, statistics, sys
for d in sorted(glob.glob(sys.argv[1] + "/*/")):
    res = {}
    for f in glob.glob(d + "**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "rt_scan_kernel" in r["Kernel_Name"]:
                res.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    med = {k: statistics.median(v) for k, v in res.items()}
    rd = med.get("FETCH_SIZE", 0) * 1024 * 2
    wr = med.get("WRITE_SIZE", 0) * 1024
    print(os.path.basename(d.rstrip("/")), "read(x2) %.3f GB write %.3f GB total %.3f GB" % (rd / 1e9, wr / 1e9, (rd + wr) / 1e9))
PY
