#!/usr/bin/env python3
"""Benchmark of the hot path: GB/s of stream scanned (+ matches/sec) on
snort.dict, one process per GPU (BASELINE.json configs 3 and 4).

A "step" is one scan of the rank's whole stream shard (default 1 GiB of
seeded synthetic ASCII, generated on the device, resident in HBM before the
timed region) through the HIP kernel, writing the dense per-position match
ids (u32; the read_block contract).  Shards are independent streams (one per
rank, distinct seeds): weak scaling, no data-path collective.  The
collectives are RCCL all-reduces of match counts, the per-pattern histogram
and the max-over-ranks time.  --layout split instead cuts ONE logical
stream of N x --bytes into rank shards (patternmatching_amd.shard.shard_plan:
each rank generates its shard plus the max_len-1 bytes before it as
context), so the all-reduced match count is that of the whole stream.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...

With --gpus N > 1 and no launcher (no WORLD_SIZE in the environment) the
process starts N ranks itself (one child process per GPU, rendezvous on
127.0.0.1) after running the CPU-baseline leg, before anything touches a
GPU.  Under a launcher WORLD_SIZE must equal --gpus.

The default run (snort, ascii, dense, rt) adds, after the timed steps, two
more measurements to the same JSON line: `count_only` (the same stream, the
RT kernel counting matches, no ids written) and `deep` (the lines stream --
the dictionary's own patterns back to back -- through the `auto` kind, with
the reference CPU loop timed on a sample of it).

Prints one JSON line on rank 0.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "GB/s stream scanned + matches/sec, snort.dict, 1/2/4/8 MI355X vs CPU ref"
DATA = os.path.join(REPO, "tests", "golden", "data")
DICTS = {"et": ["et.dict"], "snort": ["snort.dict"], "merged": ["snort.dict", "et.dict"]}
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md, HBM3E peak (spec)
WIDTH = {"dense": 4, "dense16": 2, "count": 0}  # bytes written per stream position
CAND_NAME = {0: "RT", 1: "RT", 2: "AC dense rows", 3: "AC rows + records", 4: "AC rows + records (16-B record loads)",
             5: "AC rows + records (64-B deep blocks)", 6: "AC rows + records (two chains per lane)"}
# a reference AC object per CPU-baseline process: snort's table is ~1.06 GB
# (2072 B per state, mpac.c:43-48), so the process count is also bounded by memory
REF_PROC_BYTES = 1_300_000_000


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--dict", default="snort", choices=list(DICTS))
    p.add_argument("--bytes", type=int, default=1 << 30, help="stream bytes per GPU")
    p.add_argument("--mode", default="dense", choices=list(WIDTH),
                   help="dense: u32 id per position; dense16: u16 id per position; count: match count only")
    p.add_argument("--kernel", default="rt", choices=["rt", "ac", "auto"],
                   help="rt: reverse-trie kernel; ac: the AC-DFA (dense rows or rows + records, timed); "
                        "auto: RT or the AC-DFA, picked per launch")
    p.add_argument("--stream", default="ascii", choices=["ascii", "bytes", "ship", "lines"],
                   help="ascii / bytes: seeded synthetic (DESIGN.md §6); ship: the reference's shipped "
                        "dictionaries_generated.stream tiled to --bytes (adversarial: deep matches); lines: "
                        "the dictionary's patterns drawn at random, '\\n' after each (deep, no period)")
    p.add_argument("--seed", type=int, default=1)
    p.add_argument("--layout", default="shards", choices=["shards", "split"],
                   help="shards: an independent seeded stream per rank; split: one stream of N x --bytes "
                        "cut into rank shards with max_len-1 bytes of context (ascii / bytes streams)")
    p.add_argument("--cpu-sample", type=int, default=256 << 20, help="bytes of the CPU-baseline sample")
    p.add_argument("--cpu-cores", type=int, default=0,
                   help="CPU-baseline processes (0 = the job's host-core share, bounded by memory)")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--no-extra", action="store_true", help="skip the count_only and deep measurements")
    p.add_argument("--image-cache", default="auto",
                   help="compiled-automaton cache directory (SURVEY §8f item 2): 'auto' = $PM_IMAGE_CACHE, or with "
                        "more than one rank /tmp/pm_image_cache (rank 0 compiles and writes it, the other ranks "
                        "then read it instead of compiling); 'off' = none")
    p.add_argument("--score", action="store_true",
                   help="after timing, score the ids against the AC-DFA reliable instance on the device "
                        "(measure.c:174-190) and report FP/FN/partial rates (dense mode)")
    return p.parse_args(argv)


# --------------------------------------------------------------------------
# CPU baseline (rank 0, before any GPU call)
# --------------------------------------------------------------------------

def host_share():
    """(nproc, share): the machine's CPUs and this job's share of them (the
    GPU box sets OMP_NUM_THREADS to the job's share; os.cpu_count() shows
    the whole machine)."""
    n = os.cpu_count() or 1
    share = os.environ.get("OMP_NUM_THREADS")
    s = min(n, int(share)) if share and share.isdigit() and int(share) > 0 else n
    return n, max(1, s)


def mem_available():
    try:
        with open("/proc/meminfo") as f:
            for ln in f:
                if ln.startswith("MemAvailable:"):
                    return int(ln.split()[1]) * 1024
    except OSError:
        pass
    return 16 << 30


def stream_sample(kind, dict_key, nbytes, seed):
    """The CPU sample's bytes: a seeded ascii / bytes stream or a lines
    stream of the dictionary (pm_gen_lines_dict; no device)."""
    import patternmatching_amd as pm
    if kind == "lines":
        return pm.Dictionary([os.path.join(DATA, x) for x in DICTS[dict_key]]).gen_lines(nbytes, seed)
    return pm.gen_stream(nbytes, seed, 0 if kind == "ascii" else 1)


def cpu_baseline(args, stream=None, sample_bytes=None, multi=True):
    """The reference's own per-byte AC loop (oracle/_ref/ref_driver, built from
    the reference's sources, mps_table[MPS_AC].read_char per byte): on 1 core
    over the first sample bytes of the stream, and (multi) on the job's host
    cores as one process per core, each on its own seeded sample (the
    aggregate is the sum of the per-process rates).  Beside it the C port of
    the loop (oracle/ac_oracle.c, same bytes, 1 core), so the baseline
    survives without the reference binary.  Test infrastructure, used here
    only as the measured baseline."""
    import patternmatching_amd as pm  # noqa: F401  (host library only: no device call)
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from oracle_lib import Oracle
    stream = stream or args.stream
    nbytes = sample_bytes or args.cpu_sample
    paths = [os.path.join(DATA, d) for d in DICTS[args.dict]]
    ref = os.path.join(REPO, "oracle", "_ref", "ref_driver")
    nproc, share = host_share()
    sample = f"first {nbytes} bytes of the seed-{args.seed} {stream} stream, {args.dict}.dict"
    data = stream_sample(stream, args.dict, nbytes, args.seed)
    o = Oracle(paths)
    secs, nonnull = o.time_scan(data, threads=1)
    port = {"value": round(nbytes / secs / 1e9, 6), "unit": "GB/s", "cores": 1, "seconds": round(secs, 4),
            "nonnull": nonnull, "sample": sample + "; oracle/ac_oracle.c per-byte read_char (the C port)"}
    del o
    res = {"value": port["value"], "unit": "GB/s", "cores": 1, "kind": "port", "sample": port["sample"],
           "nproc": nproc, "share": share, "port": port}
    if not os.path.exists(ref):
        return res
    try:
        with tempfile.NamedTemporaryFile(prefix="pm_cpu_", suffix=".stream", dir="/tmp", delete=False) as f:
            data.tofile(f)
            path = f.name
        try:
            r = subprocess.run([ref, "timefile", path] + paths, check=True, capture_output=True, text=True,
                               timeout=900)
        finally:
            os.unlink(path)
        one = json.loads(r.stdout)
        single = {"value": round(one["MBps"] / 1000.0, 6), "unit": "GB/s", "cores": 1, "seconds": one["seconds"],
                  "nonnull": one["nonnull"], "sample": sample}
        res.update({"value": single["value"], "cores": 1, "kind": "reference",
                    "sample": sample + "; reference Core/src objects, mps_table[MPS_AC].read_char per byte",
                    "single_core": single})
        if not multi or stream not in ("ascii", "bytes"):
            return res
        P = args.cpu_cores or min(share, max(1, mem_available() // REF_PROC_BYTES), 64)
        per = max(1 << 20, nbytes // 2)
        mode = 0 if stream == "ascii" else 1
        procs = [subprocess.Popen([ref, "time", str(args.seed + 1000 + k), str(mode), str(per)] + paths,
                                  stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True)
                 for k in range(P)]
        outs = [json.loads(p.communicate(timeout=900)[0]) for p in procs]
        agg = sum(o["MBps"] for o in outs) / 1000.0
        res.update({"value": round(agg, 6), "cores": P,
                    "sample": f"{P} concurrent processes (one per core of the {share}-core share of "
                              f"{nproc}), each the first {per} bytes of its own seeded {stream} stream (seeds "
                              f"{args.seed + 1000}..), {args.dict}.dict; reference Core/src objects, "
                              "mps_table[MPS_AC].read_char per byte; value = sum of the per-process rates",
                    "per_core_min": round(min(o["MBps"] for o in outs) / 1000.0, 6)})
    except (subprocess.SubprocessError, OSError, ValueError, KeyError) as e:
        res["reference_error"] = repr(e)[:200]
    return res


def cpu_legs(args):
    """Every CPU baseline of this run: the workload's stream, and for the
    default run's deep measurement a lines-stream sample."""
    out = {"main": cpu_baseline(args)}
    if extras_on(args):
        out["deep"] = cpu_baseline(args, stream="lines", sample_bytes=min(args.cpu_sample, 64 << 20), multi=False)
    return out


def image_cache_dir(args, world):
    """Where the ranks share the compiled automaton (None: each compiles)."""
    if args.image_cache == "off":
        return None
    if args.image_cache != "auto":
        return args.image_cache
    return os.environ.get("PM_IMAGE_CACHE") or ("/tmp/pm_image_cache" if world > 1 else None)


def compile_ordered(build, cache_dir, use_dist, rank, dist):
    """Rank 0 compiles first (writing the shared image cache), the others
    after a barrier (reading it): N ranks pay one host compile, not N.
    Each rank still uploads its own replica of the automaton to its GPU
    (replicated per GPU).  Returns build()'s value."""
    shared = use_dist and cache_dir is not None
    if shared and rank != 0:
        dist.barrier()
    v = build()
    if shared and rank == 0:
        dist.barrier()
    return v


def extras_on(args):
    return (not args.no_extra and args.stream == "ascii" and args.mode == "dense" and args.kernel == "rt"
            and args.layout == "shards")


# --------------------------------------------------------------------------
# launcher: --gpus N without torchrun
# --------------------------------------------------------------------------

def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(args):
    """Start args.gpus ranks (this script, one child process per GPU) with
    the torch.distributed environment a launcher would set.  The CPU leg runs
    here first, before any process touches a GPU, and reaches rank 0 through
    a file.  Returns the exit status (the first failing rank's)."""
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cpu_path = None
    if not args.no_cpu:
        with tempfile.NamedTemporaryFile("w", prefix="pm_bench_cpu_", suffix=".json", dir="/tmp", delete=False) as f:
            json.dump(cpu_legs(args), f)
            cpu_path = f.name
        env["PM_BENCH_CPU_JSON"] = cpu_path
    port = free_port()
    procs = []
    try:
        for r in range(args.gpus):
            e = dict(env, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                     LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
            procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=e))
        rc = 0
        pending = list(procs)
        while pending:
            for p in list(pending):
                code = p.poll()
                if code is None:
                    continue
                pending.remove(p)
                if code != 0 and rc == 0:
                    rc = code
                    for q in pending:  # a rank failed: the others would wait at a collective forever
                        q.terminate()
            time.sleep(0.2)
        return rc
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
        if cpu_path:
            os.unlink(cpu_path)


# --------------------------------------------------------------------------
# one rank
# --------------------------------------------------------------------------

def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args))
    world = int(env_world or "1")
    if env_world is not None and world != args.gpus and not (world == 1 and args.gpus == 1):
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    # CPU legs first, before this process touches the GPU (every N)
    cpu = None
    if rank == 0 and not args.no_cpu:
        path = os.environ.get("PM_BENCH_CPU_JSON")
        if path:
            with open(path) as f:
                cpu = json.load(f)
        else:
            cpu = cpu_legs(args)

    import torch
    import torch.distributed as dist

    use_dist = world > 1 or os.environ.get("PM_BENCH_DIST") == "1"
    backend = os.environ.get("PM_BENCH_BACKEND", "nccl")
    if os.environ.get("PM_BENCH_REHEARSE") == "1":
        # launcher / rendezvous rehearsal without a GPU (CPU test suite): gloo,
        # no device, placeholder timings; never a measurement.  The start-up
        # protocol runs for real on the host: rank 0 flattens the automaton
        # into the shared image cache, the others read it after the barrier
        dist.init_process_group("gloo")
        t = torch.tensor([float(rank + 1)], dtype=torch.float64)
        dist.all_reduce(t)
        startup = None
        cache_dir = image_cache_dir(args, world)
        if cache_dir is not None:
            import ctypes
            import patternmatching_amd as pm
            lib = pm.load()
            t0 = time.perf_counter()
            pats = pm.Dictionary([os.path.join(DATA, x) for x in DICTS[args.dict]]).patterns()
            arr = (ctypes.c_char_p * len(pats))(*pats)
            lens = (ctypes.c_uint32 * len(pats))(*[len(x) for x in pats])
            t1 = time.perf_counter()
            h = compile_ordered(lambda: lib.pm_flat_build_cached(arr, lens, len(pats), 1, cache_dir.encode()),
                                cache_dir, True, rank, dist)
            startup = {"dict_load_ms": round((t1 - t0) * 1e3, 2),
                       "compile_ms": round((time.perf_counter() - t1) * 1e3, 2),
                       "image_cache": "hit" if lib.pm_flat_cache_hit(h) else "miss", "image_kind": "rt (host only)"}
            lib.pm_flat_free(h)
        ranks = [None] * dist.get_world_size()
        dist.all_gather_object(ranks, {"rank": rank, "pid": os.getpid(), "startup": startup})
        if rank == 0:
            print(json.dumps({"rehearsal": True, "n_gpus": dist.get_world_size(), "world_size": dist.get_world_size(),
                              "rank_sum": t.item(), "per_rank": ranks, "image_cache_dir": cache_dir,
                              "cpu_baseline": cpu and cpu["main"]}),
                  flush=True)
        dist.destroy_process_group()
        return

    import patternmatching_amd as pm

    # one GPU per rank.  Under RCCL two ranks on one GPU would hang or fail
    # inside a collective, so a world larger than the node's GPUs is refused
    # here, before any collective; a gloo rehearsal (tests) may share one.
    ngpu = torch.cuda.device_count()
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    if use_dist and backend == "nccl" and (local_world > ngpu or local >= ngpu):
        print(f"bench.py: {local_world} ranks on this node (LOCAL_RANK {local}) but {ngpu} visible GPU(s); "
              "RCCL needs one GPU per rank (PM_BENCH_BACKEND=gloo rehearses ranks sharing a GPU)",
              file=sys.stderr, flush=True)
        sys.exit(3)
    dev = local % max(1, ngpu)
    torch.cuda.set_device(dev)
    if use_dist:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)
        assert dist.get_world_size() == world
    coll = "cuda" if backend == "nccl" else "cpu"  # gloo rehearsals reduce host tensors
    prop = torch.cuda.get_device_properties(dev)
    my_dev = {"ordinal": dev, "pci_bus_id": "%04x:%02x:%02x.0" % (prop.pci_domain_id, prop.pci_bus_id,
                                                                  prop.pci_device_id),
              "uuid": str(getattr(prop, "uuid", "")), "name": prop.name}
    devices = [my_dev]
    my_dev["host"] = socket.gethostname()
    if use_dist:
        devices = [None] * world
        dist.all_gather_object(devices, my_dev)
        # one GPU per rank: distinct (host, PCI bus id) pairs -- every node of
        # a multi-node world has its own GPUs with the same bus ids
        if backend == "nccl" and len({(d["host"], d["pci_bus_id"]) for d in devices}) != world:
            if rank == 0:
                print(f"bench.py: ranks share GPUs under RCCL: {devices}", file=sys.stderr, flush=True)
            sys.exit(3)

    def all_reduce(t, op):
        if not use_dist:
            return t
        x = t.to(coll)
        dist.all_reduce(x, op=op)
        return x.to(t.device)

    def all_gather(vals):
        if not use_dist:
            return [vals]
        x = torch.tensor(vals, dtype=torch.float64, device=coll)
        out = [torch.empty_like(x) for _ in range(world)]
        dist.all_gather(out, x)
        return [o.tolist() for o in out]

    lib = pm.load()
    lib.pm_hip_set_device(dev)
    global HBM_PEAK_GBS
    HBM_PEAK_GBS = lib.pm_hip_hbm_peak_gbs()  # the one constant the CLI's CSV prices against too

    # start-up, per rank: the device runtime's first allocation (lazy init,
    # ~150 ms, paid once per process: without it the first compile's upload
    # would carry it -- profiles/r06/startup/startup_probe.json), the
    # dictionary's parse, then compile() -- the host flatten (or the shared
    # image cache's read) and the upload of this rank's replica of the
    # automaton to its GPU
    t_i0 = time.perf_counter()
    torch.empty(1, device="cuda").zero_()
    torch.cuda.synchronize()
    init_ms = (time.perf_counter() - t_i0) * 1e3
    t_s0 = time.perf_counter()
    d = pm.Dictionary([os.path.join(DATA, x) for x in DICTS[args.dict]])
    dict_ms = (time.perf_counter() - t_s0) * 1e3
    cache_dir = image_cache_dir(args, world)
    m = pm.HipMatcher(args.kernel)
    if cache_dir:
        m.set_image_cache(cache_dir)
    m.add_dictionary(d)
    compile_ordered(m.compile, cache_dir, use_dist, rank, dist)
    cs = m.compile_stats()
    startup = {"runtime_init_ms": round(init_ms, 2), "dict_load_ms": round(dict_ms, 2),
               "compile_ms": cs["compile_ms"], "upload_ms": cs["upload_ms"],
               "image_bytes": cs["image_bytes"],
               "upload_gbps": round(cs["image_bytes"] / (cs["upload_ms"] * 1e-3) / 1e9, 2) if cs["upload_ms"] else None,
               "image_cache": ("hit" if cs["image_cache_hit"] else "miss") if cache_dir else "off",
               "wall_ms": round((time.perf_counter() - t_s0) * 1e3, 2)}
    startups = [startup]
    if use_dist:
        startups = [None] * world
        dist.all_gather_object(startups, startup)

    n = args.bytes
    stream = torch.cuda.current_stream()
    seed = args.seed + rank  # independent shard per rank
    pos0 = 0  # context bytes before the rank's first position (split layout)
    gen_off = 0
    if args.layout == "split":
        if args.stream in ("ship", "lines"):
            raise SystemExit("--layout split needs a generated stream (ascii / bytes)")
        from patternmatching_amd.shard import shard_plan
        seed = args.seed  # one logical stream
        sh = shard_plan(world * n, world, rank, lib.pm_hip_max_pattern_len(m.obj))
        ctx_lo = sh.ctx_lo & ~15  # 16-aligned: the scan starts on an aligned position
        pos0, n, gen_off = sh.lo - ctx_lo, sh.hi - sh.lo, ctx_lo
    text = torch.empty(pos0 + n + 64, dtype=torch.uint8, device="cuda")

    def fill(kind, matcher, seed_):
        if kind == "ship":
            import numpy as np
            ship = torch.from_numpy(np.fromfile(os.path.join(DATA, "dictionaries_generated.stream"), dtype=np.uint8))
            reps = (n + 64 + ship.numel() - 1) // ship.numel()
            text.copy_(ship.to("cuda").repeat(reps)[: n + 64])
        elif kind == "lines":
            matcher.gen_lines_device(text.data_ptr(), n + 64, seed_, stream.cuda_stream)
        elif lib.pm_hip_gen_stream_device(text.data_ptr(), gen_off, pos0 + n + 64, seed_,
                                          0 if kind == "ascii" else 1, stream.cuda_stream) != 0:
            raise RuntimeError(lib.pm_hip_last_error().decode())

    fill(args.stream, m, seed)
    width = WIDTH[args.mode]
    out = torch.empty(n, dtype={4: torch.int32, 2: torch.int16}[width], device="cuda") if width else None
    count = torch.zeros(1, dtype=torch.int64, device="cuda")
    out_ptr = out.data_ptr() if out is not None else None

    def timed(matcher, steps, warmup, optr, w, cnt):
        """Pick phase (ac / auto: launches synchronized one by one until the
        kind holds a choice, at most 16), W warmups, the hold pinned over the
        timed steps, then `steps` launches between synchronizations and
        barriers.  Returns (elapsed s, mean kernel ms from hipEvents on the
        launch stream, held choice)."""
        def step():
            matcher.scan_device(text.data_ptr(), 0, pos0, n, optr, cnt.data_ptr(), stream.cuda_stream,
                                out_width=w or 4)
        held = matcher.hold_choice(0)
        for _ in range(16):
            if held != -1:
                break
            step()
            torch.cuda.synchronize()
            held = matcher.hold_choice(0)
        for _ in range(warmup):
            step()
        torch.cuda.synchronize()
        held = matcher.hold_choice(steps + 1)
        if use_dist:
            dist.barrier()
        cnt.zero_()
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(steps):
            evs[k][0].record(stream)
            step()
            evs[k][1].record(stream)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        if use_dist:
            dist.barrier()
        return t1 - t0, sum(a.elapsed_time(b) for a, b in evs) / steps, held

    elapsed_mine, kernel_ms_mine, held = timed(m, args.steps, args.warmup, out_ptr, width, count)
    per_rank = all_gather([float(rank), elapsed_mine, kernel_ms_mine])
    stats = all_reduce(torch.tensor([elapsed_mine, kernel_ms_mine], dtype=torch.float64, device="cuda"),
                       dist.ReduceOp.MAX)
    torch.cuda.synchronize()
    t_cnt = time.perf_counter()
    matches = all_reduce(count.clone(), dist.ReduceOp.SUM)  # RCCL over xGMI: the match-count reduction
    torch.cuda.synchronize()
    count_ar_ms = (time.perf_counter() - t_cnt) * 1e3

    # after the timed region: all-matches (patterns ending at each position,
    # i.e. the suffix-chain length of each id), the per-pattern histogram
    # (all-reduced: SURVEY §8e) and, with --score, accuracy against the
    # reliable AC instance, all on the device
    extra = {}
    if width == 4:
        sc = torch.zeros(5, dtype=torch.int64, device="cuda")
        m.score_device(out.data_ptr(), out.data_ptr(), n, sc.data_ptr(), stream.cuda_stream)
        allm = sc.clone()
        hist = torch.zeros(lib.pm_hip_n_patterns(m.obj) + 1, dtype=torch.int64, device="cuda")
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(2):  # the second launch is timed (the first pays first-touch costs)
            hist.zero_()
            e0.record(stream)
            m.pattern_counts_device(out.data_ptr(), n, hist.data_ptr(), stream.cuda_stream)
            e1.record(stream)
            torch.cuda.synchronize()
        hist_ms = e0.elapsed_time(e1)
        t_ar = time.perf_counter()
        hist = all_reduce(hist, dist.ReduceOp.SUM)
        torch.cuda.synchronize()
        ar_ms = (time.perf_counter() - t_ar) * 1e3
        extra["pattern_counts"] = {"patterns_seen": int((hist > 0).sum().item()),
                                   "occurrences_per_step": int(hist.sum().item()),
                                   "kernel_ms": round(hist_ms, 4),
                                   "all_reduce_ms": round(ar_ms, 3) if use_dist else None,
                                   "what": "per-pattern occurrences (suffix chains of the ids) of one step, "
                                           "pm_hip_pattern_counts_device per rank, then an all-reduce (sum) of "
                                           f"{hist.numel()} u64 over ranks"}
        if args.score:
            ac = pm.HipMatcher("ac")
            ac.add_dictionary(d)
            ac.compile()
            ref = torch.empty(n, dtype=torch.int32, device="cuda")
            ac.scan_device(text.data_ptr(), 0, pos0, n, ref.data_ptr(), None, stream.cuda_stream)
            sc.zero_()
            e0.record(stream)
            m.score_device(out.data_ptr(), ref.data_ptr(), n, sc.data_ptr(), stream.cuda_stream)
            e1.record(stream)
            torch.cuda.synchronize()
            c = [int(v) for v in sc.tolist()]
            extra["accuracy"] = {"reliable": "AC-DFA (HIP)", "positions": n, "success": c[0],
                                 "false_pos_rate": c[3] / n, "false_neg_rate": c[2] / n, "partial_rate": c[1] / n,
                                 "score_ms": round(e0.elapsed_time(e1), 4)}
            del ref, ac
        allm = all_reduce(allm, dist.ReduceOp.SUM)
        extra["all_matches_per_step"] = int(allm[4].item())
    elapsed, kernel_ms = stats.tolist()
    total_matches = int(matches.item())

    # the same kernel's streaming floor, live on this GPU: rt_scan_kernel<2>
    # runs the chunk loop's loads and stores with no lookups (its ids are
    # not matches; `out` is not used after this)
    floor = None
    if rank == 0 and args.kernel == "rt" and pos0 == 0:
        fts = []
        for r in range(4):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            rc = lib.pm_hip_streaming_floor_device(m.obj, text.data_ptr(), n, out_ptr, width, stream.cuda_stream)
            e1.record(stream)
            torch.cuda.synchronize()
            if rc != 0:
                break
            if r:
                fts.append(e0.elapsed_time(e1))
        if fts:
            fms = sorted(fts)[len(fts) // 2]
            floor = {"kernel_ms": round(fms, 4), "achieved": round(n * (1 + width) / (fms * 1e-3) / 1e9, 2),
                     "kernel_over_floor": round(kernel_ms / fms, 4),
                     "what": "rt_scan_kernel<2> on this GPU: the same loads and stores, no lookups "
                             "(pm_hip_streaming_floor_device); kernel_over_floor = kernel_ms / floor kernel_ms"}

    # the default run's extra lines: count-only on the same stream, and the
    # deep lines stream through the auto kind
    count_only = deep = configs = None
    if extras_on(args):
        ksteps = min(args.steps, 10)
        cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
        _, c_ms, _ = timed(m, ksteps, 2, None, 0, cnt)
        c_ms = all_reduce(torch.tensor([c_ms], dtype=torch.float64, device="cuda"), dist.ReduceOp.MAX).item()
        c_matches = all_reduce(cnt.clone(), dist.ReduceOp.SUM).item() // ksteps
        count_only = {"kernel": "reverse-suffix-trie walk, count only (no ids written)", "stream": args.stream,
                      "steps": ksteps, "kernel_ms": round(c_ms, 4),
                      "stream_gbps": round(world * n / (c_ms * 1e-3) / 1e9, 2),
                      "matches_per_step": int(c_matches), "matches_per_sec": round(c_matches / (c_ms * 1e-3), 1),
                      "roofline": {"bound": "hbm", "achieved": round(n / (c_ms * 1e-3) / 1e9, 2),
                                   "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                   "frac": round(n / (c_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                   "algorithmic_bytes_per_launch": n}}
        del m  # the deep leg's images need the room more than this object
        ma = pm.HipMatcher("auto")
        ma.add_dictionary(d)
        ma.compile()
        fill("lines", ma, seed)
        dcnt = torch.zeros(1, dtype=torch.int64, device="cuda")
        dsteps = min(args.steps, 5)
        _, d_ms, d_held = timed(ma, dsteps, 1, out_ptr, 4, dcnt)
        d_ms = all_reduce(torch.tensor([d_ms], dtype=torch.float64, device="cuda"), dist.ReduceOp.MAX).item()
        d_matches = all_reduce(dcnt.clone(), dist.ReduceOp.SUM).item() // dsteps
        ach = n * 5 / (d_ms * 1e-3) / 1e9
        dtr = load_traffic(f"{args.dict}-lines-{n}-dense-auto")
        d_gather = gather_roofline(lib, ma, d_ms, dtr)
        deep = {"kernel": "auto kind (RT, or after a deep RT launch the faster AC-DFA form by timed trials)",
                "picked": CAND_NAME.get(d_held, str(d_held)), "stream": "lines", "mode": "dense",
                "steps": dsteps, "kernel_ms": round(d_ms, 4),
                "stream_gbps": round(world * n / (d_ms * 1e-3) / 1e9, 2),
                "matches_per_step": int(d_matches), "matches_per_sec": round(d_matches / (d_ms * 1e-3), 1),
                "data": "synthetic deep-match stream: the dictionary's own patterns drawn at random (splitmix64 "
                        "per 1 KiB block), '\\n' after each, generated in HBM (DESIGN.md §6)",
                "roofline": {"bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": round(ach / HBM_PEAK_GBS, 4), "algorithmic_bytes_per_launch": n * 5,
                             "traffic": dtr["traffic_bytes"] if dtr else None,
                             "traffic_source": dtr["source"] if dtr else None},
                "gather_roofline": d_gather,
                "cpu_baseline": cpu.get("deep") if cpu else None}
        ma.free()
        del ma
        configs = other_configs(args, pm, lib, world, all_reduce, dist, text=text, out=out)

    if rank == 0:
        last_kernel = CAND_NAME.get(held, "RT") if held > 0 else "RT" if args.kernel == "rt" else "AC"
        total_bytes = world * args.bytes * args.steps  # every rank scans --bytes positions
        value = total_bytes / elapsed / 1e9
        alg_per_pos = 1 + width  # 1 B read + the id written per position
        achieved = n * alg_per_pos / (kernel_ms * 1e-3) / 1e9
        workload_key = f"{args.dict}-{args.stream}-{n}-{args.mode}-{args.kernel}"
        tr = load_traffic(workload_key)
        traffic = tr["traffic_bytes"] if tr else None
        rates = [args.bytes * args.steps / r[1] / 1e9 for r in per_rank]
        res = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": {"ship": "the reference's shipped Streams/dictionaries_generated.stream (10,240 B) tiled in "
                             "HBM; dictionaries from the reference",
                     "lines": "synthetic deep-match stream: the dictionary's own patterns drawn at random "
                              "(splitmix64 per 1 KiB block), '\\n' after each, generated in HBM (DESIGN.md §6)"}.get(
                args.stream, "synthetic: seeded splitmix64 %s stream per GPU (DESIGN.md §6), generated in HBM; "
                             "dictionaries from the reference" % args.stream),
            "config": {
                "workload": f"{args.dict}.dict, {n} B {args.stream} stream per GPU, "
                            + {"dense": "dense u32 match id per position", "dense16": "dense u16 match id per position",
                               "count": "match count only"}[args.mode],
                "dict": args.dict,
                "stream_bytes_per_gpu": n,
                "mode": args.mode,
                "kernel": ("auto: RT, or after a deep RT launch (spill > 10%%) the fastest of RT and timed trials of "
                           "both AC-DFA forms (held: %s)" % last_kernel if args.kernel == "auto" else
                           "Aho-Corasick DFA, the faster of its two forms by timed trials (held: %s)" % last_kernel
                           if args.kernel == "ac" else "reverse-suffix-trie walk"),
                "parallelism": (f"independent stream shards x{world}" if args.layout == "shards" else
                                f"one {world * args.bytes} B stream split x{world} (max_len-1 B context per shard)"),
                "layout": args.layout,
            },
            "world_size": world,
            "per_rank": [{"rank": int(r[0]), "gbps": round(g, 3), "kernel_ms": round(r[2], 4),
                          "device": devices[int(r[0])], "startup": startups[int(r[0])]}
                         for r, g in zip(per_rank, rates)],
            "image_cache_dir": cache_dir,
            "match_count_all_reduce_ms": round(count_ar_ms, 3) if use_dist else None,
            "rank_spread": round(max(rates) / min(rates), 4),
            "matches_per_sec": round(total_matches / elapsed, 1),
            "matches_per_step": total_matches // max(1, args.steps),
            **({"all_matches_per_sec": round(extra["all_matches_per_step"] * args.steps / elapsed, 1)}
               if "all_matches_per_step" in extra else {}),
            **extra,
            "kernel_ms": round(kernel_ms, 4),
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "traffic_source": tr["source"] if tr else None,
                "algorithmic_bytes_per_launch": n * alg_per_pos,
                "streaming_floor": floor,
            },
            "cpu_baseline": cpu["main"] if cpu else None,
            **({"count_only": count_only} if count_only else {}),
            **({"deep": deep} if deep else {}),
            **({"configs": configs} if extras_on(args) else {}),
        }
        print(json.dumps(res), flush=True)
    if use_dist:
        dist.destroy_process_group()


def other_configs(args, pm, lib, world, all_reduce, dist, text, out):
    """The other BASELINE.json configs on the same kernels, per rank, timed
    like the headline (max over ranks): C2 (et.dict, 64 MiB ASCII, dense
    u32 ids), C5 (snort + et merged, 4 GiB ASCII, dense u32: one 4 GiB
    scan_device call per step, which the RT launcher runs as four 1 GiB
    kernel launches -- its queue keeps 30-bit positions), the merged
    dictionary on the deep lines stream through the auto kind, and the
    reference's own published configuration (results.csv:2-4): snort + et
    merged over its shipped Streams/dictionaries_generated.stream, tiled to
    1 GiB, through the auto kind.  The 1 GiB text and id buffers of the
    headline are reused where they are large enough.  `traffic` comes from
    profiles/traffic.json when a PMC summary of that exact workload exists
    (rocprofv3 --pmc of the equivalent single-workload bench run)."""
    import torch
    res = {}
    stream = torch.cuda.current_stream()
    rank = int(os.environ.get("RANK", "0"))

    def run(name, dict_key, kind, stream_kind, nbytes, steps):
        d = pm.Dictionary([os.path.join(DATA, x) for x in DICTS[dict_key]])
        m = pm.HipMatcher(kind)
        m.add_dictionary(d)
        m.compile()
        t = text if nbytes <= text.numel() - 64 else torch.empty(nbytes + 64, dtype=torch.uint8, device="cuda")
        o = out if nbytes <= out.numel() else torch.empty(nbytes, dtype=torch.int32, device="cuda")
        if stream_kind == "lines":
            m.gen_lines_device(t.data_ptr(), nbytes + 64, args.seed + rank, stream.cuda_stream)
        elif stream_kind == "ship":
            import numpy as np
            ship = torch.from_numpy(np.fromfile(os.path.join(DATA, "dictionaries_generated.stream"), dtype=np.uint8))
            reps = (nbytes + 64 + ship.numel() - 1) // ship.numel()
            t[: nbytes + 64].copy_(ship.to("cuda").repeat(reps)[: nbytes + 64])
        elif lib.pm_hip_gen_stream_device(t.data_ptr(), 0, nbytes + 64, args.seed + rank, 0, stream.cuda_stream):
            raise RuntimeError(lib.pm_hip_last_error().decode())
        cnt = torch.zeros(1, dtype=torch.int64, device="cuda")

        def step():
            m.scan_device(t.data_ptr(), 0, 0, nbytes, o.data_ptr(), cnt.data_ptr(), stream.cuda_stream)
        held = m.hold_choice(0)
        for _ in range(16):
            if held != -1:
                break
            step()
            torch.cuda.synchronize()
            held = m.hold_choice(0)
        step()
        torch.cuda.synchronize()
        held = m.hold_choice(steps + 1)
        cnt.zero_()
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
        for e0, e1 in evs:
            e0.record(stream)
            step()
            e1.record(stream)
        torch.cuda.synchronize()
        ms = sum(a.elapsed_time(b) for a, b in evs) / steps
        ms = all_reduce(torch.tensor([ms], dtype=torch.float64, device="cuda"), dist.ReduceOp.MAX).item()
        matches = all_reduce(cnt.clone(), dist.ReduceOp.SUM).item() // steps
        ach = nbytes * 5 / (ms * 1e-3) / 1e9
        tr = load_traffic(f"{dict_key}-{stream_kind}-{nbytes}-dense-{kind}")
        res[name] = {"dict": dict_key, "stream": stream_kind, "bytes_per_gpu": nbytes, "mode": "dense",
                     "kernel": kind + ("" if kind == "rt" else f" (held: {CAND_NAME.get(held, str(held))})"),
                     "steps": steps, "kernel_ms": round(ms, 4),
                     "stream_gbps": round(world * nbytes / (ms * 1e-3) / 1e9, 2),
                     "matches_per_step": int(matches),
                     "table_bytes": int(m.table_bytes),
                     "roofline": {"bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                  "frac": round(ach / HBM_PEAK_GBS, 4), "algorithmic_bytes_per_launch": nbytes * 5,
                                  "traffic": tr["traffic_bytes"] if tr else None,
                                  "traffic_source": tr["source"] if tr else None}}
        if kind != "rt":
            res[name]["gather_roofline"] = gather_roofline(lib, m, ms, tr)
        m.free()
        del t, o

    run("C2_et_64MiB", "et", "rt", "ascii", 64 << 20, 20)
    run("C5_merged_4GiB", "merged", "rt", "ascii", 4 << 30, 5)
    run("merged_lines_auto", "merged", "auto", "lines", min(args.bytes, 1 << 30), 5)
    run("merged_ship_auto", "merged", "auto", "ship", min(args.bytes, 1 << 30), 5)
    return res


def gather_roofline(lib, mat, kernel_ms, tr, steps=2048):
    """The DFA kernels' own bound: table gathers, not HBM bytes.  The ceiling
    is measured live, pm_hip_gather_ceiling_device over the object's own
    sparse image (the deep kernel's 1,024 lanes per CU, each chasing
    dependent 4-B loads at uniform indices; median of 3 timed launches);
    achieved = the L2 read requests of one launch (rocprofv3
    TCP_TCC_READ_REQ_sum from profiles/traffic.json: table loads and text)
    / the kernel time.  None without the image or the PMC entry."""
    import torch
    s = torch.cuda.current_stream()
    sink = torch.zeros(1, dtype=torch.int32, device="cuda")
    ncu = torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count
    ts = []
    for r in range(4):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        rc = lib.pm_hip_gather_ceiling_device(mat.obj, steps, sink.data_ptr(), s.cuda_stream)
        e1.record(s)
        torch.cuda.synchronize()
        if rc != 0:
            return None
        if r:
            ts.append(e0.elapsed_time(e1))
    ms = sorted(ts)[len(ts) // 2]
    ceiling = steps * 1024 * ncu / (ms * 1e-3) / 1e9
    req = tr.get("l2_read_requests") if tr else None
    ach = req / (kernel_ms * 1e-3) / 1e9 if req else None
    # Two different quantities side by side, named as what they are (ADVICE
    # r05): the kernel's L2 read-request rate (text loads included, LDS row
    # hits and register-held record blocks excluded) and the probe's rate of
    # dependent 4-B global loads; their ratio is an indication of headroom,
    # not a roofline fraction of one quantity
    return {"bound": "gathers", "unit": "G/s", "ceiling": round(ceiling, 2),
            "ceiling_is": "dependent uniform 4-B global loads per second (probe)",
            "l2_read_request_rate": round(ach, 2) if ach else None,
            "request_rate_over_load_ceiling": round(ach / ceiling, 4) if ach else None,
            "requests_per_launch": req, "ceiling_ms": round(ms, 4), "ceiling_loads": steps * 1024 * ncu,
            "what": "ceiling: pm_hip_gather_ceiling_device over this object's FL image (dependent uniform 4-B "
                    "loads, the kernel's launch shape); l2_read_request_rate: TCP_TCC_READ_REQ_sum per launch "
                    "(profiles/traffic.json: L1-to-L2 read requests -- table loads and ~1/16 per byte of text "
                    "loads) / kernel time.  Different units of work: their ratio is not a roofline fraction"}


def load_traffic(workload_key):
    """HBM bytes per launch from the committed rocprofv3 PMC summary, if one
    exists for this exact workload (profiles/traffic.json)."""
    path = os.path.join(REPO, "profiles", "traffic.json")
    try:
        with open(path) as f:
            return json.load(f).get(workload_key)
    except (OSError, ValueError):
        return None


if __name__ == "__main__":
    main()
