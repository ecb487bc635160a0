#!/usr/bin/env python3
"""100 KiB read_block calls (measure.c:77, 284) of ac and auto objects whose
launches run the DFA kernels (snort; random ASCII for ac, the lines stream
for auto, where its pick holds a DFA form): wall us per call, median of
REPS, gids and pattern ids.  One JSON object; run once per library build
(PM_LIBPM) to compare builds."""
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

N = 100 << 10
REPS = 200
lib = pm.load()
d = pm.Dictionary([os.path.join(REPO, "tests", "golden", "data", "snort.dict")])
res = {"bytes": N, "reps": REPS, "lib": os.environ.get("PM_LIBPM", "libpm.so")}
for kind, stream in (("ac", "ascii"), ("auto", "lines"), ("ac", "lines")):
    m = pm.HipMatcher(kind)
    m.add_dictionary(d)
    m.compile()
    if stream == "ascii":
        text = np.ascontiguousarray(pm.gen_stream(N * 8, 1, 0))
    else:
        text = np.empty(N * 8, np.uint8)
        m.lib.pm_gen_lines_host(m.obj, text.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), N * 8, 1)
    gids = np.empty(N, np.uint32)
    k = [0]

    def call():
        o = (k[0] % 8) * N
        k[0] += 1
        lib.pm_hip_read_block_gid(m.obj, text[o:o + N].ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), N,
                                  gids.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)))

    for _ in range(30):
        call()
    t = []
    for _ in range(REPS):
        t0 = time.perf_counter()
        call()
        t.append(time.perf_counter() - t0)
    res[f"{kind}_{stream}_gid_us"] = round(statistics.median(t) * 1e6, 2)
    res[f"{kind}_{stream}_last_kernel"] = int(m.lib.pm_hip_kernel_last(m.obj))
    m.free()
print(json.dumps(res))
