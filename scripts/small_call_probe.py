#!/usr/bin/env python3
"""Where a 100 KiB read_block_gid call's time goes (the
reference's chunk, measure.c:77 STREAM_BUFFER_SIZE, one read_block per chunk
at measure.c:284), each piece as its own synchronous round trip, wall
microseconds per call (median of 300, snort, RT kind, ASCII):
  round_trip_empty   a one-element device op + stream synchronize: launch
                     and completion latency alone
  kernel_hbm         scan_device on HBM-resident text into HBM ids + sync
                     (the small kernel's own time plus that latency)
  kernel_zc          the same reading pinned host text and writing pinned
                     host ids (zero copy: what a small read_block launches)
  graph_zc           kernel_zc captured once into a HIP graph, then replayed
  write_zc_400k      a device copy of 400 KB into pinned host memory + sync
                     (the link's share: the ids a call brings back)
  read_block_gid     the whole call (staging, launch, wait, result copy);
                     _events: with the per-call timing events (host_events)
  read_block_ids     the same for pattern ids (read_block; ac kind too)
  host_copy_400k     memcpy of 400 KB pinned -> pageable on the host
  read_block_gid_serve0/1  the whole call with a launch per call (0) or
                     through the object's resident server grid (1, the
                     default for rt objects), with the host path's breakdown
Prints one JSON object."""
import ctypes
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import patternmatching_amd as pm  # noqa: E402

N = 100 << 10
REPS = 300
lib = pm.load()
d = pm.Dictionary([os.path.join(REPO, "tests", "golden", "data", "snort.dict")])
m = pm.HipMatcher("rt")
m.add_dictionary(d)
m.compile()
text = pm.gen_stream(N + 4096, 1, 0)
s = torch.cuda.Stream()
sp = s.cuda_stream


def timeit(fn, reps=REPS):
    for _ in range(20):
        fn()
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        t.append(time.perf_counter() - t0)
    return round(statistics.median(t) * 1e6, 2)


res = {"chunk_bytes": N, "reps": REPS}
one = torch.zeros(1, device="cuda")


def empty():
    with torch.cuda.stream(s):
        one.add_(1)
    s.synchronize()


res["round_trip_empty_us"] = timeit(empty)
dt = torch.from_numpy(np.concatenate([text, np.zeros(64, np.uint8)])).cuda()
dout = torch.empty(N, dtype=torch.int32, device="cuda")


def kernel_hbm():
    m.scan_device(dt.data_ptr(), 0, 4096, N, dout.data_ptr(), None, sp)
    s.synchronize()


res["kernel_hbm_us"] = timeit(kernel_hbm)
ht = torch.from_numpy(np.concatenate([text, np.zeros(64, np.uint8)])).pin_memory()
hout = torch.empty(N, dtype=torch.int32).pin_memory()


def kernel_zc():
    m.scan_device(ht.data_ptr(), 0, 4096, N, hout.data_ptr(), None, sp)
    s.synchronize()


res["kernel_zc_us"] = timeit(kernel_zc)
ref = dout.cpu().numpy()
assert np.array_equal(hout.numpy(), ref)
m.prepare_capture()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=s):
    m.scan_device(ht.data_ptr(), 0, 4096, N, hout.data_ptr(), None, sp)
hout.zero_()


def graph_zc():
    with torch.cuda.stream(s):  # (replay() launches on the current stream)
        g.replay()
    s.synchronize()


res["graph_zc_us"] = timeit(graph_zc)
assert np.array_equal(hout.numpy(), ref)
dsrc = torch.empty(N, dtype=torch.int32, device="cuda")


def write_zc():
    with torch.cuda.stream(s):
        hout.copy_(dsrc, non_blocking=True)
    s.synchronize()


res["write_zc_400k_us"] = timeit(write_zc)
gids = np.empty(N, np.uint32)
part = np.ascontiguousarray(text[4096:4096 + N])


def call():
    lib.pm_hip_read_block_gid(m.obj, part.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), N,
                              gids.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)))


ids = np.empty(N, np.uint64)


def call_ids(mm):
    return lambda: lib.pm_hip_read_block(mm.obj, part.ctypes.data_as(ctypes.c_char_p), N,
                                         ids.ctypes.data_as(ctypes.POINTER(ctypes.c_void_p)))


# the resident server grid (host_serve) against a launch per call, and the
# host path's breakdown of each (staging, enqueue, wait, result copy)
for sv in (0, 1):
    assert m.set_option("host_serve", sv) == 0
    m.reset()
    res[f"read_block_gid_serve{sv}_us"] = timeit(call)
    m.reset()
    res[f"read_block_ids_serve{sv}_us"] = timeit(call_ids(m))
    m.reset()
    lib.pm_hip_host_profile(1, None)
    for _ in range(REPS):
        call()
    prof = (ctypes.c_double * 5)()
    lib.pm_hip_host_profile(0, prof)
    res[f"read_block_gid_serve{sv}_breakdown_us"] = {
        k: round(prof[i] / max(prof[4], 1) * 1e6, 2) for i, k in enumerate(("stage", "enqueue", "wait", "copy"))}
    res[f"read_block_gid_serve{sv}_GBps"] = round(N / res[f"read_block_gid_serve{sv}_us"] / 1e3, 3)
for g16 in (1, 0):  # u16 gids over the link through the server
    assert m.set_option("host_gid16", g16) == 0
    m.reset()
    res[f"read_block_gid_serve1_gid16_{g16}_us"] = timeit(call)
m.set_option("host_gid16", -1)
outs = []
for sv in (0, 1):  # the same ids either way, calls carrying state
    assert m.set_option("host_serve", sv) == 0
    m.reset()
    got = []
    for _ in range(4):
        call()
        got.append(gids.copy())
    outs.append(np.concatenate(got))
assert np.array_equal(outs[0], outs[1])
m.set_option("host_serve", -1)
res["serve_stats"] = m.serve_stats()
ac = pm.HipMatcher("ac")
ac.add_dictionary(d)
ac.compile()
for ev, tag in ((0, ""), (1, "_events")):
    for mm, kname in ((m, ""), (ac, "_ac")):
        assert mm.set_option("host_events", ev) == 0
        mm.reset()
        fn = call if mm is m else (lambda: lib.pm_hip_read_block_gid(
            ac.obj, part.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), N,
            gids.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))))
        res[f"read_block_gid{kname}{tag}_us"] = timeit(fn)
        mm.reset()
        res[f"read_block_ids{kname}{tag}_us"] = timeit(call_ids(mm))
        mm.set_option("host_events", -1)
    res[f"read_block_gid{tag}_GBps"] = round(N / res[f"read_block_gid{tag}_us"] / 1e3, 3)
for g16 in (1, 0):  # u16 gids over the link, widened on the host pool
    assert m.set_option("host_gid16", g16) == 0
    m.reset()
    res[f"read_block_gid_gid16_{g16}_us"] = timeit(call)
m.set_option("host_gid16", -1)
dst = np.empty(N, np.int32)
hn = hout.numpy()
res["host_copy_400k_us"] = timeit(lambda: np.copyto(dst, hn))
print(json.dumps(res))
