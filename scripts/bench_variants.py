#!/usr/bin/env python3
"""Ablation timing of the RT kernel variants, interleaved rounds in one
process (guide §5.4 rule 24).  Prints a JSON summary."""
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
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--stream", type=int, default=0, help="0 ascii, 1 bytes, 2 the shipped stream tiled, 3 lines")
ap.add_argument("--variants", default="0,1,2")
ap.add_argument("--modes", default="dense,dense16,count")
ap.add_argument("--exact", default="", help="variants whose dense u32 ids must equal v0's (checked after timing)")
ap.add_argument("--blocks", type=int, default=0, help="RT workgroups per launch (pm_hip_debug_rt_blocks; 0 = one per CU)")
ap.add_argument("--counts", action="store_true", help="report each variant's match count of one launch (count mode)")
args = ap.parse_args()
DICTS = {"et": ["et.dict"], "snort": ["snort.dict"], "merged": ["snort.dict", "et.dict"]}
WIDTH = {"dense": 4, "dense16": 2, "count": 0}
data = os.path.join(REPO, "tests", "golden", "data")
lib = pm.load()
lib.pm_hip_debug_rt_blocks(args.blocks)
d = pm.Dictionary([os.path.join(data, x) for x in DICTS[args.dict]])
m = pm.HipMatcher("rt")
m.add_dictionary(d)
m.compile()
n = args.bytes
s = torch.cuda.current_stream()
text = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
if args.stream == 3:
    m.gen_lines_device(text.data_ptr(), n + 64, 1, s.cuda_stream)
elif args.stream == 2:
    import numpy as np
    ship = torch.from_numpy(np.fromfile(os.path.join(data, "dictionaries_generated.stream"), dtype=np.uint8))
    text.copy_(ship.cuda().repeat((n + 64) // ship.numel() + 1)[: n + 64])
else:
    lib.pm_hip_gen_stream_device(text.data_ptr(), 0, n + 64, 1, args.stream, s.cuda_stream)
out = torch.empty(n, dtype=torch.int32, device="cuda")
cnt = torch.zeros(8, dtype=torch.int64, device="cuda")
variants = [(int(v), mode) for v in args.variants.split(",") for mode in args.modes.split(",")]
times = {k: [] for k in variants}
for r in range(args.rounds + 1):
    for (v, mode) in variants:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        rc = lib.pm_hip_debug_scan_variant(m.obj, v, text.data_ptr(), n, out.data_ptr() if mode != "count" else None,
                                           WIDTH[mode], cnt.data_ptr(), s.cuda_stream)
        assert rc == 0
        e1.record(s)
        torch.cuda.synchronize()
        if r:
            times[(v, mode)].append(e0.elapsed_time(e1))
res = {}
for (v, mode), t in times.items():
    ms = statistics.median(t)
    res[f"v{v}-{mode}"] = {"ms": round(ms, 4), "min": round(min(t), 4), "GBps_stream": round(n / ms / 1e6, 1),
                           "alg_GBps": round(n * (1 + WIDTH[mode]) / ms / 1e6, 1)}
if args.counts:
    for v in sorted({v for v, _ in variants}):
        c1 = torch.zeros(1, dtype=torch.int64, device="cuda")
        assert lib.pm_hip_debug_scan_variant(m.obj, v, text.data_ptr(), n, None, 0, c1.data_ptr(), s.cuda_stream) == 0
        torch.cuda.synchronize()
        res[f"v{v}-count-matches"] = int(c1.item())
if args.exact:
    def ids(v):
        o = torch.zeros(n, dtype=torch.int32, device="cuda")
        assert lib.pm_hip_debug_scan_variant(m.obj, v, text.data_ptr(), n, o.data_ptr(), 4, cnt.data_ptr(),
                                             s.cuda_stream) == 0
        torch.cuda.synchronize()
        return o
    ref = ids(0)
    for v in (int(x) for x in args.exact.split(",")):
        res[f"v{v}-ids-equal-v0"] = bool(torch.equal(ids(v), ref))
print(json.dumps(res, indent=1))
