#!/usr/bin/env python3
"""Copy one gpu_round.sh session (gpurun_out/round_TAG) into profiles/:
the bench lines, the rocprofv3 kernel stats of the default bench, the PMC
traffic summary, the GPU test log, and profiles/traffic.json (which bench.py
reads for roofline.traffic).  Usage: collect_round.py TAG [round, e.g. r02]."""
import json
import os
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1]
rnd = sys.argv[2] if len(sys.argv) > 2 else "r01"
dst = os.path.join(REPO, "profiles", rnd)
src = os.path.join(REPO, "gpurun_out", f"round_{tag}")
os.makedirs(dst, exist_ok=True)
names = {"dense": "C3 snort 1 GiB dense_u32 (bench default, 16-core reference baseline)",
         "dense16": "snort 1 GiB dense_u16", "count": "snort 1 GiB count_only",
         "ac": "snort 1 GiB AC-DFA (reliable instance; the faster of its two forms, timed), dense_u32",
         "c2_et64m": "C2 et 64 MiB dense_u32", "c5_merged4g": "C5 merged 4 GiB dense_u32",
         "score": "snort 1 GiB dense_u32 + on-device accuracy scoring vs the AC instance (--score)",
         "ship": "snort, the shipped stream tiled to 1 GiB (deep matches), dense_u32",
         "ship_count": "snort, the shipped stream tiled to 1 GiB, count_only",
         "ship_ac": "snort, the shipped stream tiled to 1 GiB, AC-DFA (forms timed), dense_u32",
         "ship_auto": "snort, the shipped stream tiled to 1 GiB, auto kind (RT, then timed AC forms after a spilling launch), dense_u32",
         "lines": "snort, the lines stream (random dictionary patterns, no period), 1 GiB, RT, dense_u32",
         "lines_ac": "snort, the lines stream, 1 GiB, AC-DFA (forms timed: rows + records), dense_u32",
         "lines_auto": "snort, the lines stream, 1 GiB, auto kind, dense_u32"}
lines = {}
for k, label in names.items():
    p = os.path.join(src, f"bench_{k}.json")
    if os.path.exists(p):
        lines[label] = json.loads(open(p).read().strip().splitlines()[-1])
lines["_session"] = f"scripts/gpu_round.sh {tag}; one MI355X box, one call"
json.dump(lines, open(os.path.join(dst, f"bench_{rnd}.json"), "w"), indent=1)
shutil.copy(os.path.join(src, "prof", "bench_kernel_stats.csv"),
            os.path.join(dst, "rt_dense_snort_1GiB_kernel_stats.csv"))
shutil.copy(os.path.join(src, "pytest_gpu.log"), os.path.join(dst, f"pytest_gpu_{rnd}.log"))
la = os.path.join(src, "prof_lines_ac", "bench_kernel_stats.csv")
if os.path.exists(la):
    shutil.copy(la, os.path.join(dst, "ac_lines_snort_1GiB_kernel_stats.csv"))
pmc = json.load(open(os.path.join(src, "pmc_summary.json")))
json.dump(pmc, open(os.path.join(dst, "rt_dense_snort_1GiB_pmc_traffic.json"), "w"), indent=1)
tr_path = os.path.join(REPO, "profiles", "traffic.json")
tr = json.load(open(tr_path))
key = "snort-ascii-1073741824-dense-rt"
rd = pmc["FETCH_SIZE"] * 1024
wr = pmc["WRITE_SIZE"] * 1024
tr[key].update({"read_bytes_raw": rd, "read_bytes_corrected": 2 * rd, "write_bytes": wr,
                "traffic_bytes": 2 * rd + wr, "session": f"gpu_round.sh {tag}",
                "source": f"profiles/{rnd}/rt_dense_snort_1GiB_pmc_traffic.json (rocprofv3 --pmc, one counter per pass, "
                          "median over dispatches of rt_scan_kernel; 1 dispatch per 1 GiB step)"})
json.dump(tr, open(tr_path, "w"), indent=1)
for label, d in lines.items():
    if not label.startswith("_"):
        print(f"{label}: {d['value']} GB/s, kernel {d['kernel_ms']} ms, frac {d['roofline']['frac']}")
print("traffic", (2 * rd + wr) / 1e9, "GB per launch")
