#!/usr/bin/env python3
"""Shortest-segment sweep of the AC-DFA kernel (pm_hip_debug_dfa_min_seg)
over launch sizes, snort, dense u32, random ASCII or the shipped stream
tiled; every setting's ids must equal the default's.  Timing tool only;
prints one line per (size, min_seg) and a JSON summary."""
import argparse
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import patternmatching_amd as pm  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--dict", default="snort")
ap.add_argument("--stream", default="ascii", choices=["ascii", "ship"])
ap.add_argument("--sizes", default="102400,1048576,16777216,67108864,1073741824")
ap.add_argument("--min-segs", default="2048,1024,512,256,128,64")
ap.add_argument("--rounds", type=int, default=5)
args = ap.parse_args()
DICTS = {"et": ["et.dict"], "snort": ["snort.dict"], "merged": ["snort.dict", "et.dict"]}
data = os.path.join(REPO, "tests", "golden", "data")
lib = pm.load()
d = pm.Dictionary([os.path.join(data, x) for x in DICTS[args.dict]])
m = pm.HipMatcher("ac")
m.add_dictionary(d)
m.compile()
sizes = [int(x) for x in args.sizes.split(",")]
nmax = max(sizes)
s = torch.cuda.current_stream()
text = torch.empty(nmax + 64, dtype=torch.uint8, device="cuda")
if args.stream == "ascii":
    lib.pm_hip_gen_stream_device(text.data_ptr(), 0, nmax + 64, 1, 0, s.cuda_stream)
else:
    ship = torch.from_numpy(np.fromfile(os.path.join(data, "dictionaries_generated.stream"), dtype=np.uint8))
    reps = (nmax + 64 + ship.numel() - 1) // ship.numel()
    text.copy_(ship.to("cuda").repeat(reps)[: nmax + 64])
out = torch.empty(nmax, dtype=torch.int32, device="cuda")
cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
segs = [int(x) for x in args.min_segs.split(",")]
res = {}
for n in sizes:
    ref = None
    for ms_ in segs:
        lib.pm_hip_debug_dfa_min_seg(ms_)
        ts = []
        for r in range(args.rounds + 1):
            cnt.zero_()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            m.scan_device(text.data_ptr(), 0, 0, n, out.data_ptr(), cnt.data_ptr(), s.cuda_stream)
            e1.record(s)
            torch.cuda.synchronize()
            if r:
                ts.append(e0.elapsed_time(e1))
        if ref is None:
            ref = out[:n].clone()
        same = bool(torch.equal(out[:n], ref))
        ms = statistics.median(ts)
        res[f"{n}/{ms_}"] = {"ms": round(ms, 4), "GBps": round(n / ms / 1e6, 2), "same_ids": same}
        print(n, ms_, res[f"{n}/{ms_}"], flush=True)
    lib.pm_hip_debug_dfa_min_seg(0)
print(json.dumps(res))
