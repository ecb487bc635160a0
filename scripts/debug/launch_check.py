#!/usr/bin/env python3
"""One small launch per sparse-DFA variant (1 MiB of the lines stream, snort,
dense u32), each checked and synchronized before the next; stops at the first
failure and says which.  Debug tool."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
import torch  # noqa: E402
import patternmatching_amd as pm  # noqa: E402

lib = pm.load()
d = pm.Dictionary([os.path.join(REPO, "tests", "golden", "data", "snort.dict")])
m = pm.HipMatcher("ac")
m.add_dictionary(d)
m.compile()
lib.pm_hip_debug_dfa_sparse(1)
n = int(os.environ.get("N", 1 << 20))
s = torch.cuda.current_stream()
text = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
m.gen_lines_device(text.data_ptr(), n + 64, 1, s.cuda_stream)
out = torch.empty(n, dtype=torch.int32, device="cuda")
ref = None
for v in [int(x) for x in sys.argv[1].split(",")]:
    lib.pm_hip_debug_dfa_lds(v)
    out.zero_()
    torch.cuda.synchronize()
    rc = lib.pm_hip_scan_device(m.obj, text.data_ptr(), 0, 0, n, out.data_ptr(), None, s.cuda_stream)
    print("variant", v, "launch rc", rc, lib.pm_hip_last_error().decode() if rc else "", flush=True)
    if rc:
        sys.exit(1)
    torch.cuda.synchronize()
    if ref is None:
        ref = out.clone()
    print("variant", v, "ok, equal to first:", bool(torch.equal(ref, out)), flush=True)
