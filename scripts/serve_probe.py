#!/usr/bin/env python3
"""read_block at the reference's 100 KiB chunks (measure.c:77, 284) through
an rt object's resident server grid ("host_serve" 1) against a launch per
call (0), side by side in one process: wall us per call (median of REPS),
the host path's breakdown (staging, enqueue, wait, result copy / map) and,
for gids, with u16 gids over the link ("host_gid16").  The ids of both paths
are checked equal over calls that carry state.  Prints one JSON object
(PM_SERVE_BLOCKS sets the grid's workgroups)."""
import ctypes
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import patternmatching_amd as pm  # noqa: E402

N = int(os.environ.get("SERVE_PROBE_BYTES", 100 << 10))
REPS = 300
lib = pm.load()
KIND = os.environ.get("SERVE_PROBE_KIND", "rt")  # or "auto" (random ASCII: its pick holds RT)
m = pm.HipMatcher(KIND)
m.add_dictionary(pm.Dictionary([os.path.join(REPO, "tests", "golden", "data", "snort.dict")]))
m.compile()
if os.environ.get("SERVE_PROBE_STREAM") == "lines":  # deep: the lines stream
    part = np.empty(N, np.uint8)
    m.lib.pm_gen_lines_host(m.obj, part.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), N, 1)
else:
    part = np.ascontiguousarray(pm.gen_stream(N, 1, 0))
gids = np.empty(N, np.uint32)
ids = np.empty(N, np.uint64)


def call():
    lib.pm_hip_read_block_gid(m.obj, part.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), N,
                              gids.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)))


def call_ids():
    lib.pm_hip_read_block(m.obj, part.ctypes.data_as(ctypes.c_char_p), N, ids.ctypes.data_as(ctypes.POINTER(ctypes.c_void_p)))


def timeit(fn):
    for _ in range(20):
        fn()
    t = []
    for _ in range(REPS):
        t0 = time.perf_counter()
        fn()
        t.append(time.perf_counter() - t0)
    return round(statistics.median(t) * 1e6, 2)


res = {"bytes": N, "reps": REPS, "kind": KIND, "stream": os.environ.get("SERVE_PROBE_STREAM", "ascii"),
       "serve_blocks_env": os.environ.get("PM_SERVE_BLOCKS")}
for sv in (0, 1, 0, 1):
    assert m.set_option("host_serve", sv) == 0
    for g16 in (0, 1):
        assert m.set_option("host_gid16", g16) == 0
        m.reset()
        res.setdefault(f"gid_serve{sv}_gid16_{g16}_us", []).append(timeit(call))
    m.set_option("host_gid16", -1)
    m.reset()
    res.setdefault(f"ids_serve{sv}_us", []).append(timeit(call_ids))
    m.reset()
    lib.pm_hip_host_profile(1, None)
    for _ in range(REPS):
        call()
    prof = (ctypes.c_double * 5)()
    lib.pm_hip_host_profile(0, prof)
    res[f"gid_serve{sv}_breakdown_us"] = {
        k: round(prof[i] / max(prof[4], 1) * 1e6, 2) for i, k in enumerate(("stage", "enqueue", "wait", "copy"))}
outs = []
for sv in (0, 1):
    assert m.set_option("host_serve", sv) == 0
    m.reset()
    got = []
    for _ in range(4):
        call()
        got.append(gids.copy())
    outs.append(np.concatenate(got))
assert np.array_equal(outs[0], outs[1])
res["serve_stats"] = m.serve_stats()
res["gid_GBps"] = {k: round(N / min(v) / 1e3, 3) for k, v in res.items() if isinstance(v, list) and k.startswith("gid_serve")}
print(json.dumps(res))
