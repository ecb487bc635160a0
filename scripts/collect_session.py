#!/usr/bin/env python3
"""Copy one scripts/gpu_round4.sh session (gpurun_out/TAG) into
profiles/ROUND/session_TAG -- the bench lines, the rocprofv3 kernel stats of
each leg, the PMC summaries, the GPU test and smoke logs -- and update
profiles/traffic.json, which bench.py reads for roofline.traffic: the
headline kernel (rt_scan_kernel, C3) and the deep leg's kernel (the lines
stream through the auto kind).  Usage: collect_session.py TAG ROUND."""
import glob
import json
import os
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag, rnd = sys.argv[1], sys.argv[2]
src = os.path.join(REPO, "gpurun_out", tag)
dst = os.path.join(REPO, "profiles", rnd, f"session_{tag}")
os.makedirs(dst, exist_ok=True)
for name in ("bench.json", "bench_prof.json", "bench_prof_count.json", "bench_prof_deep.json", "pmc_summary.json",
             "pmc_deep_summary.json", "pytest_gpu.log", "smoke.log", "ref_loop_per_byte_rate.json"):
    p = os.path.join(src, name)
    if os.path.exists(p):
        shutil.copy(p, os.path.join(dst, name))
for leg, out in (("prof", "rt_dense_snort_1GiB_kernel_stats.csv"), ("prof_count", "rt_count_snort_1GiB_kernel_stats.csv"),
                 ("prof_deep", "auto_lines_snort_1GiB_kernel_stats.csv")):
    f = glob.glob(os.path.join(src, leg, "**", "*kernel_stats.csv"), recursive=True)
    if f:
        shutil.copy(f[0], os.path.join(dst, out))

tr_path = os.path.join(REPO, "profiles", "traffic.json")
tr = json.load(open(tr_path))
rel = os.path.relpath(dst, REPO)
pmc = json.load(open(os.path.join(src, "pmc_summary.json")))
rd, wr = pmc["FETCH_SIZE"] * 1024, pmc["WRITE_SIZE"] * 1024
tr["snort-ascii-1073741824-dense-rt"].update({
    "read_bytes_raw": rd, "read_bytes_corrected": 2 * rd, "write_bytes": wr, "traffic_bytes": 2 * rd + wr,
    "session": f"gpu_round4.sh {tag}",
    "source": f"{rel}/pmc_summary.json (rocprofv3 --pmc, one counter per pass, median over dispatches of "
              "rt_scan_kernel<0, 4, false>; 1 dispatch per 1 GiB step)"})
p = os.path.join(src, "pmc_deep_summary.json")
if os.path.exists(p):
    d = json.load(open(p))
    drd, dwr = d["FETCH_SIZE"] * 1024, d["WRITE_SIZE"] * 1024
    tr["snort-lines-1073741824-dense-auto"] = {
        "source": f"{rel}/pmc_deep_summary.json (rocprofv3 --pmc, one counter per pass, median over dispatches of "
                  "the sparse AC-DFA kernel the auto kind holds on the lines stream, dfa_sparse_stage16_kernel<88, 4>; "
                  "1 dispatch per 1 GiB step)",
        "read_bytes_raw": drd, "write_bytes": dwr, "traffic_bytes": drd + dwr,
        "algorithmic_bytes": (1 << 30) * 5,
        "note": "FETCH_SIZE (KiB) x1024, not doubled: this kernel's reads are gathers of table lines, each L2 miss "
                "one 64-B request (TCC_MISS x 64 B = FETCH_SIZE on the lines stream, profiles/r04/measure_r04a); "
                "the x2 correction of MI355X_MICROARCH.md is calibrated for 16 B/lane streams.  WRITE_SIZE exact "
                "for the id stores.  Traffic well above the algorithmic 5 B per position = the table gathers "
                "(the automaton's rows and records do not fit L2)",
        "session": f"gpu_round4.sh {tag}"}
json.dump(tr, open(tr_path, "w"), indent=1)
b = json.load(open(os.path.join(src, "bench.json")))
print("C3", b["value"], b["kernel_ms"], b["roofline"]["frac"], "count", b["count_only"]["kernel_ms"],
      "deep", b["deep"]["kernel_ms"], "configs", {k: v["kernel_ms"] for k, v in b.get("configs", {}).items()})
print("traffic C3", (2 * rd + wr) / 1e9, "GB; deep", tr.get("snort-lines-1073741824-dense-auto", {}).get("traffic_bytes"))
