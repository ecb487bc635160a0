#!/usr/bin/env python3
"""Start-up cost of compile() in one process: the same dictionary compiled by
successive objects (rt, then auto, then rt again), with and without the
image cache -- separates the process's first device allocations from the
flatten and the upload themselves.  Prints one JSON object."""
import json
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import patternmatching_amd as pm  # noqa: E402

DATA = os.path.join(REPO, "tests", "golden", "data")
lib = pm.load()
lib.pm_hip_set_device(0)
d = pm.Dictionary([os.path.join(DATA, "snort.dict")])
cache = tempfile.mkdtemp(prefix="pm_cache_")
res = []
for kind, use_cache in (("rt", False), ("rt", False), ("auto", False), ("rt", True), ("rt", True), ("auto", True),
                        ("auto", True)):
    t0 = time.perf_counter()
    m = pm.HipMatcher(kind)
    if use_cache:
        m.set_image_cache(cache)
    m.add_dictionary(d)
    m.compile()
    st = m.compile_stats()
    st.update({"kind": kind, "cache": use_cache, "wall_ms": round((time.perf_counter() - t0) * 1e3, 2),
               "upload_gbps": round(st["image_bytes"] / (st["upload_ms"] * 1e-3) / 1e9, 2) if st["upload_ms"] else None})
    res.append(st)
    m.free()
print(json.dumps(res))
