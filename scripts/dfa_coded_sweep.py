#!/usr/bin/env python3
"""Form (dense rows / sparse rows + records) and launch shape of the
output-coded AC-DFA kernel: lanes per CU
(pm_hip_debug_dfa_shape) x segments per lane (pm_hip_debug_dfa_chains),
snort, dense u32, on random ASCII, the shipped stream tiled and the lines
stream; every shape's ids must equal the first one's.  Timing tool only."""
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
ap.add_argument("--lanes", default="256,512,1024")
ap.add_argument("--streams", default="ascii,ship,lines")
ap.add_argument("--forms", default="0,1", help="0 = dense rows, 1 = sparse rows + records (pm_hip_debug_dfa_sparse)")
ap.add_argument("--chains", default="1,2")
ap.add_argument("--blocks", default="32", help="sparse form, one chain: positions per block (16,32)")
ap.add_argument("--width", type=int, default=4, choices=[2, 4], help="id width of the timed launches")
ap.add_argument("--dense-blocks", default="0", help="dense form: positions per block (16,32; 0 = default)")
ap.add_argument("--variants", default="0", help="sparse form, one chain: kernel variants (pm_hip_debug_dfa_variant)")
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
ref = torch.empty(n, dtype=torch.int32 if args.width == 4 else torch.int16, device="cuda")
out = torch.empty_like(ref)
res = {}


def timed(fn):
    ts = []
    for r in range(args.rounds + 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        fn()
        e1.record(s)
        torch.cuda.synchronize()
        if r:
            ts.append(e0.elapsed_time(e1))
    return statistics.median(ts)


for stream in args.streams.split(","):
    if stream == "ascii":
        lib.pm_hip_gen_stream_device(text.data_ptr(), 0, n + 64, 1, 0, s.cuda_stream)
    elif stream == "lines":
        m.gen_lines_device(text.data_ptr(), n + 64, 1, s.cuda_stream)
    else:
        ship = torch.from_numpy(np.fromfile(os.path.join(data, "dictionaries_generated.stream"), dtype=np.uint8))
        text.copy_(ship.cuda().repeat((n + 64) // ship.numel() + 1)[: n + 64])
    first = True
    for form in [int(x) for x in args.forms.split(",")]:
        lib.pm_hip_debug_dfa_sparse(form)
        for lanes in [int(x) for x in args.lanes.split(",")]:
            lib.pm_hip_debug_dfa_shape(lanes)
            for ch in [int(x) for x in args.chains.split(",")]:
                lib.pm_hip_debug_dfa_chains(ch)
                combos = [(b, v) for b in map(int, args.blocks.split(",")) for v in map(int, args.variants.split(","))]
                dcombos = [(b, v) for b in map(int, args.dense_blocks.split(",")) for v in map(int, args.variants.split(","))]
                for blk, var in combos if form and ch == 1 else dcombos:
                    lib.pm_hip_debug_dfa_block(blk)
                    lib.pm_hip_debug_dfa_variant(var)
                    dst = ref if first else out
                    ms = timed(lambda: m.scan_device(text.data_ptr(), 0, 0, n, dst.data_ptr(), None, s.cuda_stream,
                                                     out_width=args.width))
                    same = True if first else bool(torch.equal(out, ref))
                    first = False
                    key = f"{stream}/{'sparse' if form else 'dense'}/L{lanes}/ch{ch}/b{blk}/v{var}"
                    res[key] = {"ms": round(ms, 4), "GBps": round(n / ms / 1e6, 1), "same": same}
                    print(key, res[key], flush=True)
lib.pm_hip_debug_dfa_shape(0)
lib.pm_hip_debug_dfa_chains(0)
lib.pm_hip_debug_dfa_sparse(-1)
lib.pm_hip_debug_dfa_block(0)
lib.pm_hip_debug_dfa_variant(0)
print(json.dumps(res))
