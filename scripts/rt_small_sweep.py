#!/usr/bin/env python3
"""The reverse-trie kernel at small launch sizes: the one-thread-per-position
kernel (rt_small_kernel) against the chunked product kernel, ids checked
equal, snort, ASCII and the lines stream, u32 ids.  Prints one JSON object."""
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402
import patternmatching_amd as pm  # noqa: E402

lib = pm.load()
d = pm.Dictionary([os.path.join(REPO, "tests", "golden", "data", "snort.dict")])
m = pm.HipMatcher("rt")
m.add_dictionary(d)
m.compile()
s = torch.cuda.current_stream()
N = 16 << 20
res = {}
for stream in ("ascii", "lines"):
    text = torch.empty(N + 64, dtype=torch.uint8, device="cuda")
    if stream == "lines":
        m.gen_lines_device(text.data_ptr(), N + 64, 3, s.cuda_stream)
    else:
        lib.pm_hip_gen_stream_device(text.data_ptr(), 0, N + 64, 3, 0, s.cuda_stream)
    for n in (16 << 10, 100 << 10, 256 << 10, 1 << 20, 4 << 20, N - 4096):
        outs, ts = {}, {}
        for mode, lim in (("chunked", 0), ("small", 1 << 40)):
            m.set_option("rt_small_max", lim)
            o = torch.zeros(n, dtype=torch.int32, device="cuda")
            t = []
            for r in range(12):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                m.scan_device(text.data_ptr(), 0, 4096, n, o.data_ptr(), None, s.cuda_stream)
                e1.record(s)
                torch.cuda.synchronize()
                if r >= 2:
                    t.append(e0.elapsed_time(e1) * 1e3)
            outs[mode], ts[mode] = o, statistics.median(t)
        m.set_option("rt_small_max", -1)
        assert torch.equal(outs["chunked"], outs["small"]), (stream, n)
        res[f"{stream}-{n}"] = {"chunked_us": round(ts["chunked"], 2), "small_us": round(ts["small"], 2)}
print(json.dumps(res, indent=1))
