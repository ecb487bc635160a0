#!/usr/bin/env python3
"""Summarise a gpu_round5.sh session directory: per leg, the dominant scan
kernel's rocprofv3 average duration (--stats) and its PMC traffic per
bench step (FETCH_SIZE / WRITE_SIZE medians over its dispatches x the
dispatches one step makes; for the DFA legs also TCP_TCC_READ_REQ_sum, the
L2 read requests bench.py sets against its live gather ceiling).  Writes <dir>/legs.json; with --traffic FILE
also merges the legs into profiles/traffic.json's format (FILE), citing
--cite (the directory the session is committed under)."""
import argparse
import csv
import glob
import json
import os
import statistics

LEGS = {  # leg -> (bench workload key, dispatches of the scan kernel per step)
    "c3": ("snort-ascii-1073741824-dense-rt", 1),
    "count": ("snort-ascii-1073741824-count-rt", 1),
    "deep": ("snort-lines-1073741824-dense-auto", 1),
    "c2": ("et-ascii-67108864-dense-rt", 1),
    "c5": ("merged-ascii-4294967296-dense-rt", 4),
    "merged_lines": ("merged-lines-1073741824-dense-auto", 1),
    "merged_ship": ("merged-ship-1073741824-dense-auto", 1),
}
ALG = {"dense": 5, "count": 1, "dense16": 3}
SCAN = ("rt_scan_kernel", "dfa_", "rt_small_kernel")


def is_scan(name):
    return any(k in name for k in SCAN) and "variant" not in name


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--traffic", default="")
    ap.add_argument("--cite", default="")
    a = ap.parse_args()
    legs = {}
    for leg, (key, per_step) in LEGS.items():
        stats = glob.glob(os.path.join(a.dir, f"prof_{leg}", "**", "*kernel_stats.csv"), recursive=True)
        if not stats:
            continue
        rows = [r for f in stats for r in csv.DictReader(open(f)) if is_scan(r["Name"])]
        if not rows:
            continue
        # the held kernel: the scan kernel with the most dispatches (the auto
        # kind's measured RT launch and DFA trials run once or twice)
        top = max(rows, key=lambda r: int(r["Calls"]))
        name = top["Name"]
        ent = {"kernel": name, "calls": int(top["Calls"]), "avg_ms": float(top["AverageNs"]) / 1e6, "workload": key,
               "dispatches_per_step": per_step}
        pmc = {}
        for f in glob.glob(os.path.join(a.dir, f"pmc_{leg}", "*", "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if r["Kernel_Name"] == name:
                    pmc.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
        med = {k: statistics.median(v) for k, v in pmc.items()}
        ent["pmc_median_per_dispatch"] = med
        if "FETCH_SIZE" in med and "WRITE_SIZE" in med:
            raw = med["FETCH_SIZE"] * 1024 * per_step
            # the gfx950 x2 read correction (MI355X_MICROARCH.md §HBM) is
            # calibrated for streaming loads: applied to the RT kernels'
            # text stream, not to the DFA kernels' table gathers (each L2
            # miss one 64-B request)
            rt = "rt_" in name
            rd = raw * 2 if rt else raw
            wr = med["WRITE_SIZE"] * 1024 * per_step
            mode = key.split("-")[3]
            n = int(key.split("-")[2])
            ent.update({"read_bytes_raw": raw, "read_bytes_corrected": rd, "write_bytes": wr,
                        "traffic_bytes": rd + wr, "algorithmic_bytes": n * ALG[mode]})
        if "TCP_TCC_READ_REQ_sum" in med:  # L2 read requests (the DFA kernels' gathers + text)
            ent["l2_read_requests"] = med["TCP_TCC_READ_REQ_sum"] * per_step
        legs[leg] = ent
    json.dump(legs, open(os.path.join(a.dir, "legs.json"), "w"), indent=1)
    for leg, e in legs.items():
        print(f"{leg:13s} {e['kernel'][:64]:64s} calls {e['calls']:3d} avg {e['avg_ms']:.4f} ms "
              f"traffic {e.get('traffic_bytes', 0) / 1e9:.2f} GB (alg {e.get('algorithmic_bytes', 0) / 1e9:.2f})")
    if a.traffic:
        tr = json.load(open(a.traffic)) if os.path.exists(a.traffic) else {}
        for leg, e in legs.items():
            if "traffic_bytes" not in e:
                continue
            tr[e["workload"]] = {
                "source": f"{a.cite or a.dir}/legs.json (rocprofv3 --pmc, one counter per pass, median over the "
                          f"dispatches of {e['kernel']}; {e['dispatches_per_step']} dispatch(es) per bench step)",
                "read_bytes_raw": e["read_bytes_raw"], "read_bytes_corrected": e["read_bytes_corrected"],
                "write_bytes": e["write_bytes"], "traffic_bytes": e["traffic_bytes"],
                "algorithmic_bytes": e["algorithmic_bytes"],
                **({"l2_read_requests": e["l2_read_requests"]} if "l2_read_requests" in e else {}),
                "note": "FETCH_SIZE (KiB) x1024 (x2 for the RT kernels' streaming text reads, MI355X_MICROARCH.md "
                        "§HBM; not for the DFA kernels' table gathers), WRITE_SIZE x1024; per bench step",
                "session": os.path.basename(a.dir.rstrip("/"))}
        json.dump(tr, open(a.traffic, "w"), indent=1)


if __name__ == "__main__":
    main()
