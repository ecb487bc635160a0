#!/usr/bin/env python3
"""Steady-state cost of the auto kind's re-measurement: LAUNCHES scan_device
launches of 256 MiB of a deep stream through `auto` with nothing pinned
(no pm_hip_hold_choice), one synchronize at the end; prints the mean ms
per launch and the share of RT launches (each one a measurement).  With
PM_LIBPM naming another build, the same for it (scripts/build_ab.sh)."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import patternmatching_amd as pm  # noqa: E402

LAUNCHES = int(os.environ.get("LAUNCHES", "600"))
SYNC = int(os.environ.get("SYNC", "0"))  # 1: synchronize after every launch (a read_block-like caller)
n = 256 << 20
res = {"lib": os.environ.get("PM_LIBPM", "libpm.so"), "launches": LAUNCHES, "bytes": n, "sync": SYNC}
for stream in ("lines", "ship"):
    d = pm.Dictionary([os.path.join(REPO, "tests", "golden", "data", "snort.dict")])
    m = pm.HipMatcher("auto")
    m.add_dictionary(d)
    m.compile()
    s = torch.cuda.current_stream()
    dt = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    if stream == "lines":
        m.gen_lines_device(dt.data_ptr(), n + 64, 3, s.cuda_stream)
    else:
        ship = np.fromfile(os.path.join(REPO, "tests", "golden", "data", "dictionaries_generated.stream"), np.uint8)
        dt.copy_(torch.from_numpy(np.tile(ship, (n + 64) // len(ship) + 1)[: n + 64]).cuda())
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    for _ in range(3):
        m.scan_device(dt.data_ptr(), 0, 0, n, out.data_ptr(), None, s.cuda_stream)
    torch.cuda.synchronize()
    rt = 0
    t0 = time.perf_counter()
    for _ in range(LAUNCHES):
        m.scan_device(dt.data_ptr(), 0, 0, n, out.data_ptr(), None, s.cuda_stream)
        rt += m.kernel_last == pm.KIND_RT
        if SYNC:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    res[stream] = {"ms_per_launch": round((time.perf_counter() - t0) * 1e3 / LAUNCHES, 4), "rt_launches": rt}
    m.free()
    del dt, out
print(json.dumps(res))
