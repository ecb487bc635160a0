#!/usr/bin/env python3
"""PCIe-inclusive rate of the host-buffer boundary (read_block from host
memory, MEASUREMENTS.md §5): times pm_hip_read_block_gid / pm_hip_read_block over a
host stream in fixed-size calls, and the drop-in CLI end to end on a stream
file.  Prints one JSON object."""
import ctypes
import json
import os
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import patternmatching_amd as pm  # noqa: E402

DATA = os.path.join(REPO, "tests", "golden", "data")
n = int(os.environ.get("PM_HOST_BYTES", 1 << 30))
chunk = int(os.environ.get("PM_HOST_CHUNK", 16 << 20))
text = pm.gen_stream(n, 1, 0)
d = pm.Dictionary([os.path.join(DATA, "snort.dict")])
res = {"stream_bytes": n, "chunk_bytes": chunk}
for kind in ("rt", "ac"):
    m = pm.HipMatcher(kind)
    m.add_dictionary(d)
    m.compile()
    gids = np.empty(chunk, np.uint32)
    ids = (ctypes.c_void_p * chunk)()
    lib = m.lib
    # warm-up: the first call allocates the pipeline's pinned slots
    lib.pm_hip_read_block_gid(m.obj, text.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), chunk,
                              gids.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)))
    for api in ("gid", "ids"):
        lib.pm_hip_reset(m.obj)
        t0 = time.perf_counter()
        for off in range(0, n, chunk):
            part = text[off:off + chunk]
            if api == "gid":
                lib.pm_hip_read_block_gid(m.obj, part.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), len(part),
                                          gids.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)))
            else:
                lib.pm_hip_read_block(m.obj, part.ctypes.data_as(ctypes.c_char_p), len(part), ids)
        dt = time.perf_counter() - t0
        res[f"{kind}_read_block_{api}_GBps"] = round(n / dt / 1e9, 3)
    # -1 = unmeasured: small calls are untimed unless the "host_events"
    # option is on (include/pm_hip.h), and timing them costs ~7 us a call
    dev_s = lib.pm_hip_device_seconds(m.obj)
    res[f"{kind}_device_seconds"] = round(dev_s, 4) if dev_s >= 0 else None

# raw PCIe copy rates between pinned host memory and HBM (the host path moves
# 1 B up and 4 B (gid) down per position)
import torch  # noqa: E402
for name, nb in (("h2d", 256 << 20), ("d2h", 1 << 30)):
    h = torch.empty(nb, dtype=torch.uint8, pin_memory=True)
    dv = torch.empty(nb, dtype=torch.uint8, device="cuda")
    for r in range(4):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        (dv.copy_(h, non_blocking=True) if name == "h2d" else h.copy_(dv, non_blocking=True))
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    res[f"pcie_{name}_GBps"] = round(nb / dt / 1e9, 2)

# the CLI end to end: two GPU matchers + the reliable instance + scoring
with tempfile.TemporaryDirectory() as td:
    sp = os.path.join(td, "x.stream")
    text[: 64 << 20].tofile(sp)
    out = os.path.join(td, "res.csv")
    t0 = time.perf_counter()
    r = subprocess.run([pm.CLI_PATH, "-d", os.path.join(DATA, "snort.dict"), "-s", sp, "-o", out, "-B", str(chunk)],
                       capture_output=True, text=True, timeout=600)
    res["cli_seconds_64MiB"] = round(time.perf_counter() - t0, 3)
    res["cli_rc"] = r.returncode
    res["cli_csv"] = open(out).read().strip().split("\n") if r.returncode == 0 else r.stderr[-500:]
print(json.dumps(res, indent=1))
