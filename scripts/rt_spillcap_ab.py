#!/usr/bin/env python3
"""Side by side, one process: the RT kernel with its per-wave spill region
capped at 1-16 chunks ("spill_cap_chunks", include/pm_hip.h) -- a smaller
region makes the wave resolve its candidates (the tail's batched probes and
walks) several times inside the chunk loop, where other waves' streaming
hides the probes' latency, instead of once after it, when every wave of the
CU waits at the same time.  1 GiB per stream, count only and u32 ids;
counts (and ids) checked equal across caps.  Prints one JSON object."""
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
ap.add_argument("--rounds", type=int, default=7)
ap.add_argument("--streams", default="ascii,ship,lines")
ap.add_argument("--caps", default="0,8,4,2,1")
ap.add_argument("--modes", default="count,dense")
args = ap.parse_args()
DICTS = {"et": ["et.dict"], "snort": ["snort.dict"], "merged": ["snort.dict", "et.dict"]}
data = os.path.join(REPO, "tests", "golden", "data")
lib = pm.load()
m = pm.HipMatcher("rt")
m.add_dictionary(pm.Dictionary([os.path.join(data, x) for x in DICTS[args.dict]]))
m.compile()
n = args.bytes
s = torch.cuda.current_stream()
text = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
out = torch.empty(n, dtype=torch.int32, device="cuda")
cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
res = {"dict": args.dict, "bytes": n}
for st in args.streams.split(","):
    if st == "lines":
        m.gen_lines_device(text.data_ptr(), n + 64, 1, s.cuda_stream)
    elif st == "ship":
        ship = torch.from_numpy(np.fromfile(os.path.join(data, "dictionaries_generated.stream"), dtype=np.uint8))
        text.copy_(ship.cuda().repeat((n + 64) // ship.numel() + 1)[: n + 64])
    else:
        lib.pm_hip_gen_stream_device(text.data_ptr(), 0, n + 64, 1, 0, s.cuda_stream)
    for mode in args.modes.split(","):
        caps = [int(c) for c in args.caps.split(",")]
        times = {c: [] for c in caps}
        counts = {}
        ref = None
        for r in range(args.rounds + 1):
            for c in caps:
                assert m.set_option("spill_cap_chunks", c) == 0
                cnt.zero_()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                m.scan_device(text.data_ptr(), 0, 0, n, out.data_ptr() if mode == "dense" else None, cnt.data_ptr(),
                              s.cuda_stream)
                e1.record(s)
                torch.cuda.synchronize()
                if r:
                    times[c].append(e0.elapsed_time(e1))
                counts[c] = int(cnt.item())
                if r == 0 and mode == "dense":
                    if ref is None:
                        ref = out.clone()
                    elif not torch.equal(ref, out):
                        raise SystemExit(f"{st}: ids differ at cap {c}")
        del ref
        assert len(set(counts.values())) == 1, counts
        for c in caps:
            res[f"{st}-{mode}-cap{c}"] = {"ms": round(statistics.median(times[c]), 4), "matches": counts[c]}
print(json.dumps(res))
