#!/usr/bin/env python3
"""Per-call breakdown of the read_block host path at the reference's chunk
size (measure.c:77 STREAM_BUFFER_SIZE = 100 KiB; measure.c:284 read_block per
chunk): staging, enqueue (copies + launch), wait, result copy / id map, in
microseconds per call (pm_hip_host_profile), and the rate, for the rt
and ac kinds, gids and pattern ids.  PM_HOST_VARIANTS (e.g. "ev,evspin")
repeats it per setting of the object's host options (pm_hip_set_option):
the spin wait ("spin": host_spin), u16 gids for small gid calls ("g16":
host_gid16), the per-call timing events ("ev": host_events; device_us is
-1 without them) and the host pool off ("pool0": host_pool), side by
side.  Prints one JSON object."""
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import patternmatching_amd as pm  # noqa: E402

DATA = os.path.join(REPO, "tests", "golden", "data")
n = int(os.environ.get("PM_HOST_BYTES", 64 << 20))
chunk = int(os.environ.get("PM_HOST_CHUNK", 100 << 10))
text = pm.gen_stream(n, 1, 0)
d = pm.Dictionary([os.path.join(DATA, "snort.dict")])
res = {"stream_bytes": n, "chunk_bytes": chunk, "PM_HOST_ZC": os.environ.get("PM_HOST_ZC", "default 3")}
lib = pm.load()
prof = (ctypes.c_double * 5)()
variants = os.environ.get("PM_HOST_VARIANTS", "")
for var, kind in [(v, k) for v in (variants.split(",") if variants else [""])
                  for k in os.environ.get("PM_HOST_KINDS", "rt,ac").split(",")]:
    m = pm.HipMatcher(kind)
    m.add_dictionary(d)
    m.compile()
    if var:
        m.set_option("host_spin", 1 if "spin" in var else 0)
        m.set_option("host_gid16", 1 if "g16" in var else 0)
        m.set_option("host_events", 1 if "ev" in var else 0)
        m.set_option("host_pool", 0 if "pool0" in var else -1)
    gids = np.empty(chunk, np.uint32)
    ids = (ctypes.c_void_p * chunk)()
    lib.pm_hip_read_block_gid(m.obj, text.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), chunk,
                              gids.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)))
    for api in ("gid", "ids"):
        lib.pm_hip_reset(m.obj)
        for rep in range(2):  # the second pass is reported
            lib.pm_hip_host_profile(1, None)
            t0 = time.perf_counter()
            for off in range(0, n, chunk):
                part = text[off:off + chunk]
                if api == "gid":
                    lib.pm_hip_read_block_gid(m.obj, part.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), len(part),
                                              gids.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)))
                else:
                    lib.pm_hip_read_block(m.obj, part.ctypes.data_as(ctypes.c_char_p), len(part), ids)
            dt = time.perf_counter() - t0
            lib.pm_hip_host_profile(0, prof)
        calls = max(1.0, prof[4])
        res[f"{kind}_{api}" + (f"_{var}" if var else "")] = {"GBps": round(n / dt / 1e9, 3), "us_per_call": round(dt / calls * 1e6, 2),
                                "stage_us": round(prof[0] / calls * 1e6, 2),
                                "enqueue_us": round(prof[1] / calls * 1e6, 2),
                                "wait_us": round(prof[2] / calls * 1e6, 2),
                                "result_us": round(prof[3] / calls * 1e6, 2),
                                "device_us": round(lib.pm_hip_device_seconds(m.obj) / calls * 1e6, 2)}
    m.free()
print(json.dumps(res, indent=1))
