#!/usr/bin/env python3
"""Launch-shape sweep of the AC-DFA kernel (segments in flight per CU),
snort 1 GiB ascii, dense u32; every shape's ids must equal the first one's.
Timing tool only; prints a JSON summary."""
import argparse
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402
import patternmatching_amd as pm  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--dict", default="snort")
ap.add_argument("--bytes", type=int, default=1 << 30)
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--lanes", default="128,256,384,512,768,1024")
args = ap.parse_args()
DICTS = {"et": ["et.dict"], "snort": ["snort.dict"], "merged": ["snort.dict", "et.dict"]}
data = os.path.join(REPO, "tests", "golden", "data")
lib = pm.load()
d = pm.Dictionary([os.path.join(data, x) for x in DICTS[args.dict]])
m = pm.HipMatcher("ac")
m.add_dictionary(d)
m.compile()
n = args.bytes
s = torch.cuda.current_stream()
text = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
lib.pm_hip_gen_stream_device(text.data_ptr(), 0, n + 64, 1, 0, s.cuda_stream)
out = torch.empty(n, dtype=torch.int32, device="cuda")
ref = None
cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
shapes = [int(x) for x in args.lanes.split(",")]
res = {}
for L in shapes:
    lib.pm_hip_debug_dfa_shape(L)
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
        ref = out.clone()
        same = True
    else:
        same = bool(torch.equal(out, ref))
    ms = statistics.median(ts)
    res[str(L)] = {"ms": round(ms, 3), "GBps_stream": round(n / ms / 1e6, 1), "nonnull": int(cnt.item()),
                       "same_ids": same}
    print(L, res[str(L)], flush=True)
lib.pm_hip_debug_dfa_shape(0)
print(json.dumps(res))
