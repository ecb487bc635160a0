#!/usr/bin/env python3
"""Debug aid: the sparse-form kernels against the RT ids on a short window
of the lines stream (the failing case of test_sparse_dfa_kernel_variants_agree),
printing the mismatching positions per kernel, warm-up rule and width."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import patternmatching_amd as pm  # noqa: E402

d = pm.Dictionary([os.path.join(REPO, "tests", "golden", "data", "snort.dict")])
rt = pm.HipMatcher("rt")
rt.add_dictionary(d)
rt.compile()
ac = pm.HipMatcher("ac")
ac.add_dictionary(d)
ac.compile()
n = 1 << 20
s = torch.cuda.current_stream().cuda_stream
dt = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
rt.gen_lines_device(dt.data_ptr(), n + 64, 11, s)
ref = torch.empty(n, dtype=torch.int32, device="cuda")
rt.scan_device(dt.data_ptr(), 0, 0, n, ref.data_ptr(), None, s)
ac.set_option("dfa_form", 2)
for size, start in ((777, 4096), (100 << 10, 12336), (4096, 0), (65536, 8192)):
    for sk in (1, 2):
        for sync in (0, 1):
            ac.set_option("sparse_kernel", sk)
            ac.set_option("dfa_sync", sync)
            a = torch.full((size,), -1, dtype=torch.int32, device="cuda")
            c = torch.zeros(2, dtype=torch.int64, device="cuda")
            h = torch.zeros(size, dtype=torch.int16, device="cuda")
            ac.scan_device(dt.data_ptr(), 0, start, size, a.data_ptr(), c[0:1].data_ptr(), s)
            ac.scan_device(dt.data_ptr(), 0, start, size, 0, c[1:2].data_ptr(), s)
            k4 = ac.sparse_kernel_last
            ac.scan_device(dt.data_ptr(), 0, start, size, h.data_ptr(), None, s, out_width=2)
            k2 = ac.sparse_kernel_last
            torch.cuda.synchronize()
            r = ref[start:start + size].cpu().numpy()
            av = a.cpu().numpy()
            hv = h.cpu().numpy().astype(np.int64) & 0xFFFF
            bad4 = np.nonzero(av != r)[0]
            bad2 = np.nonzero(hv != r)[0]
            print(c.tolist(), int((r != 0).sum()), size, start, "sk", sk, "sync", sync, "k4", k4, "bad4", len(bad4), bad4[:40].tolist(),
                  "k2", k2, "bad2", len(bad2), bad2[:40].tolist(), flush=True)
            if len(bad4):
                print("   a  ", av[bad4[:12]].tolist(), "\n   ref", r[bad4[:12]].tolist(), flush=True)
