#!/usr/bin/env python3
"""Chains in flight for the sparse AC-DFA form: kernel form
(pm_hip_debug_dfa_lds: 0 = plain, 2 = register record blocks, 5 / 6 = the
latter with two segments per lane, 32 / 16-position blocks) x lanes per CU
(pm_hip_debug_dfa_shape), snort, 1 GiB, dense u32 ids (or --width 2 / 0).
One process, rounds interleaved across the settings; every setting's ids
must equal the first one's.  Timing tool only.  Prints one JSON object."""
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
ap.add_argument("--bytes", type=int, default=1 << 30)
ap.add_argument("--rounds", type=int, default=4)
ap.add_argument("--streams", default="lines")
ap.add_argument("--forms", default="2,5,6,0")
ap.add_argument("--lanes", default="512,1024,1536,2048")
ap.add_argument("--width", type=int, default=4, choices=[0, 2, 4])
ap.add_argument("--sparse", type=int, default=1, help="1: the sparse form (forms/lanes apply); 0: dense rows")
ap.add_argument("--sync", default="1", help="warm-ups from synchronizing 3-grams (pm_hip_debug_dfa_sync), e.g. 1,0")
args = ap.parse_args()
DICTS = {"et": ["et.dict"], "snort": ["snort.dict"], "merged": ["snort.dict", "et.dict"]}
data = os.path.join(REPO, "tests", "golden", "data")
lib = pm.load()
d = pm.Dictionary([os.path.join(data, x) for x in DICTS[args.dict]])
m = pm.HipMatcher("ac")
m.add_dictionary(d)
m.compile()
lib.pm_hip_debug_dfa_sparse(args.sparse)
n = args.bytes
w = args.width
s = torch.cuda.current_stream()
text = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
ref = torch.empty(n * max(w, 1) // 4 + 16, dtype=torch.int32, device="cuda")
out = torch.empty_like(ref)
cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
res = {}
settings = [(f, l, y) for f in map(int, args.forms.split(",")) for l in map(int, args.lanes.split(","))
            for y in map(int, args.sync.split(","))]
for st in args.streams.split(","):
    if st == "lines":
        m.gen_lines_device(text.data_ptr(), n + 64, 1, s.cuda_stream)
    elif st == "ship":
        ship = torch.from_numpy(np.fromfile(os.path.join(data, "dictionaries_generated.stream"), dtype=np.uint8))
        text.copy_(ship.cuda().repeat((n + 64) // ship.numel() + 1)[: n + 64])
    else:
        lib.pm_hip_gen_stream_device(text.data_ptr(), 0, n + 64, 1, 0, s.cuda_stream)
    times = {k: [] for k in settings}
    counts = {}
    for r in range(args.rounds + 1):
        for k in settings:
            f, lanes, y = k
            lib.pm_hip_debug_dfa_lds(f)
            lib.pm_hip_debug_dfa_shape(lanes)
            lib.pm_hip_debug_dfa_sync(y)
            cnt.zero_()
            dst = ref if k == settings[0] else out
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            m.scan_device(text.data_ptr(), 0, 0, n, dst.data_ptr() if w else None, cnt.data_ptr(), s.cuda_stream,
                          out_width=w or 4)
            e1.record(s)
            torch.cuda.synchronize()
            if r:
                times[k].append(e0.elapsed_time(e1))
            counts[k] = int(cnt.item())
            if r == 0 and w and k != settings[0] and not torch.equal(out, ref):
                raise SystemExit(f"{st}: form {f} lanes {lanes} sync {y}: ids differ from {settings[0]}")
    assert len(set(counts.values())) == 1, counts
    for k in settings:
        ms = statistics.median(times[k])
        res[f"{st}-f{k[0]}-L{k[1]}-y{k[2]}"] = {"ms": round(ms, 4), "stream_gbps": round(n / ms / 1e6, 1)}
        print(f"{st} form {k[0]} lanes/CU {k[1]} sync {k[2]}: {ms:.3f} ms", flush=True)
lib.pm_hip_debug_dfa_lds(-1)
lib.pm_hip_debug_dfa_shape(0)
lib.pm_hip_debug_dfa_sync(-1)
lib.pm_hip_debug_dfa_sparse(-1)
print(json.dumps(res))
