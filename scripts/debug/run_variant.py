"""Run one RT kernel variant a few times on a 1 GiB stream (profiling driver)."""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
import torch
import patternmatching_amd as pm
var, mode, stream = int(sys.argv[1]), sys.argv[2], sys.argv[3]
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 3
data = os.path.join(REPO, "tests", "golden", "data")
lib = pm.load()
d = pm.Dictionary([os.path.join(data, "snort.dict")])
m = pm.HipMatcher("rt"); m.add_dictionary(d); m.compile()
n = 1 << 30
s = torch.cuda.current_stream()
text = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
if stream == "ship":
    ship = torch.from_numpy(np.fromfile(os.path.join(data, "dictionaries_generated.stream"), dtype=np.uint8))
    text.copy_(ship.cuda().repeat((n + 64) // ship.numel() + 1)[: n + 64])
else:
    lib.pm_hip_gen_stream_device(text.data_ptr(), 0, n + 64, 1, 0, s.cuda_stream)
W = {"dense": 4, "dense16": 2, "count": 0}[mode]
out = torch.empty(n * max(W, 1) // 4 + 16, dtype=torch.int32, device="cuda")
cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
for _ in range(reps):
    assert lib.pm_hip_debug_scan_variant(m.obj, var, text.data_ptr(), n, out.data_ptr() if W else None, W,
                                         cnt.data_ptr(), s.cuda_stream) == 0
torch.cuda.synchronize()
print("ok", var, mode, stream, int(cnt.item()))
