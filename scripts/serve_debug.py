#!/usr/bin/env python3
"""Small read_block calls of an rt object through the resident server grid
(debugging aid for the host_serve path; SERVE_DEBUG_BYTES per call, default
10,000): prints each call's time and the serve stats."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import patternmatching_amd as pm  # noqa: E402

m = pm.HipMatcher("rt")
m.add_dictionary(pm.Dictionary([os.path.join(REPO, "tests", "golden", "data", "et.dict")]))
m.compile()
text = pm.gen_stream(int(os.environ.get("SERVE_DEBUG_BYTES", 10000)), 1, 0)
assert m.set_option("host_serve", 0) == 0
ref = m.read_block_gids(text)
m.reset()
assert m.set_option("host_serve", 1) == 0
t0 = time.perf_counter()
got = m.read_block_gids(text)
print("first call s", time.perf_counter() - t0, m.serve_stats(), flush=True)
assert np.array_equal(got, ref)
for k in range(5):
    m.reset()
    t0 = time.perf_counter()
    got = m.read_block_gids(text)
    print("call s", time.perf_counter() - t0, np.array_equal(got, ref), m.serve_stats(), flush=True)
m.free()
print("freed", flush=True)
