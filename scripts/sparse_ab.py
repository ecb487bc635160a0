#!/usr/bin/env python3
"""Side by side, one process: the sparse AC-DFA form's kernels (the
per-object "sparse_kernel" option, include/pm_hip.h: 1 fallback-linked,
2 lock-step 8-B units, 3 lock-step 16-B records) on 1 GiB of each stream, ids checked equal across kernels.
With PM_LIBPM naming another build of the library (scripts/build_ab.sh, e.g.
an ablation build with -DPM_FL_SPEC=2) the same for that build: run it once
per build (scripts/ab_libs.sh alternates them).  Prints one JSON object."""
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
ap.add_argument("--kernels", default="1,2")
ap.add_argument("--modes", default="dense")
args = ap.parse_args()
DICTS = {"et": ["et.dict"], "snort": ["snort.dict"], "merged": ["snort.dict", "et.dict"]}
WIDTH = {"dense": 4, "dense16": 2, "count": 0}
data = os.path.join(REPO, "tests", "golden", "data")
lib = pm.load()
d = pm.Dictionary([os.path.join(data, x) for x in DICTS[args.dict]])
m = pm.HipMatcher("ac")
m.add_dictionary(d)
m.compile()
assert m.set_option("dfa_form", 2) == 0  # the sparse form on every launch
n = args.bytes
s = torch.cuda.current_stream()
text = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
outs = {w: torch.empty(n * max(w, 1) // 4 + 16, dtype=torch.int32, device="cuda") for w in (4, 2)}
cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
res = {"lib": os.environ.get("PM_LIBPM", "libpm.so"), "dict": args.dict, "bytes": n}
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
        ks = args.kernels.split(",")
        times = {k: [] for k in ks}
        ran = {}
        ref = None
        counts = {}
        for r in range(args.rounds + 1):
            for k in ks:
                kk, hold, chains, lanes = (k.split(":") + ["", "", ""])[:4]  # kernel[:fl_hold[:fl_chains[:fl_lanes]]]
                assert m.set_option("sparse_kernel", int(kk)) == 0
                assert m.set_option("fl_hold", int(hold or 0)) == 0
                assert m.set_option("fl_chains", int(chains or 1)) == 0
                if lanes:  # (an ablation build's option)
                    assert m.set_option("fl_lanes", int(lanes)) == 0
                cnt.zero_()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                m.scan_device(text.data_ptr(), 0, 0, n, outs[w or 4].data_ptr() if w else None, cnt.data_ptr(),
                              s.cuda_stream, out_width=w or 4)
                e1.record(s)
                torch.cuda.synchronize()
                ran[k] = m.sparse_kernel_last
                if r:
                    times[k].append(e0.elapsed_time(e1))
                counts[k] = int(cnt.item())
                if r == 0 and w:
                    if ref is None:
                        ref = outs[w][: n * w // 4].clone()
                    elif not torch.equal(ref, outs[w][: n * w // 4]):
                        raise SystemExit(f"{st} {mode}: kernel {k} ids differ from kernel {ks[0]}")
        del ref
        assert len(set(counts.values())) <= 1, counts
        for k in ks:
            ms = statistics.median(times[k])
            res[f"{st}-{mode}-k{k}"] = {"ms": round(ms, 4), "stream_gbps": round(n / ms / 1e6, 1),
                                       "matches": counts[k], "ran": ran[k]}
print(json.dumps(res))
