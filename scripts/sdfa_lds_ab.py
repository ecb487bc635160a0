#!/usr/bin/env python3
"""Side by side, one process: the sparse AC-DFA form's kernels (0 = plain
dfa_sparse_kernel, 1 = LDS rows + register record blocks, 2 = record blocks
only) on 1 GiB of each stream, dense u32 / u16 / count; ids checked equal.
Prints one JSON object."""
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
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--streams", default="lines,ship,ascii")
ap.add_argument("--variants", default="0,1,2")
ap.add_argument("--modes", default="dense")
ap.add_argument("--nocheck", default="", help="timing ablations whose ids are not checked")
args = ap.parse_args()
DICTS = {"et": ["et.dict"], "snort": ["snort.dict"], "merged": ["snort.dict", "et.dict"]}
WIDTH = {"dense": 4, "dense16": 2, "count": 0}
data = os.path.join(REPO, "tests", "golden", "data")
lib = pm.load()
d = pm.Dictionary([os.path.join(data, x) for x in DICTS[args.dict]])
m = pm.HipMatcher("ac")
m.add_dictionary(d)
m.compile()
lib.pm_hip_debug_dfa_sparse(1)  # the sparse form on every launch
n = args.bytes
s = torch.cuda.current_stream()
text = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
outs = {w: torch.empty(n * max(w, 1) // 4 + 16, dtype=torch.int32, device="cuda") for w in (4, 2)}
cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
res = {}
for st in args.streams.split(","):
    if st == "lines":
        m.gen_lines_device(text.data_ptr(), n + 64, 1, s.cuda_stream)
    elif st == "ship":
        ship = torch.from_numpy(np.fromfile(os.path.join(data, "dictionaries_generated.stream"), dtype=np.uint8))
        text.copy_(ship.cuda().repeat((n + 64) // ship.numel() + 1)[: n + 64])
    else:
        lib.pm_hip_gen_stream_device(text.data_ptr(), 0, n + 64, 1, 0 if st == "ascii" else 1, s.cuda_stream)
    for mode in args.modes.split(","):
        w = WIDTH[mode]
        vs = [int(v) for v in args.variants.split(",")]
        times = {v: [] for v in vs}
        ref = None
        counts = {}
        for r in range(args.rounds + 1):
            for v in vs:
                lib.pm_hip_debug_dfa_lds(v)
                cnt.zero_()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                m.scan_device(text.data_ptr(), 0, 0, n, outs[w or 4].data_ptr() if w else None, cnt.data_ptr(),
                              s.cuda_stream, out_width=w or 4)
                e1.record(s)
                torch.cuda.synchronize()
                if r:
                    times[v].append(e0.elapsed_time(e1))
                counts[v] = int(cnt.item())
                if r == 0 and w and str(v) not in args.nocheck.split(","):
                    h = int(outs[w][: n * w // 4].view(torch.int64)[:: 997].sum().item())
                    if ref is None:
                        ref = (h, outs[w][: n * w // 4].clone())
                    elif not torch.equal(ref[1], outs[w][: n * w // 4]):
                        raise SystemExit(f"{st} {mode}: variant {v} ids differ from variant {vs[0]}")
        del ref
        assert len({c for v, c in counts.items() if str(v) not in args.nocheck.split(",")}) <= 1, counts
        for v in vs:
            ms = statistics.median(times[v])
            res[f"{st}-{mode}-v{v}"] = {"ms": round(ms, 4), "stream_gbps": round(n / ms / 1e6, 1),
                                       "matches": counts[v]}
print(json.dumps(res))
