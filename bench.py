#!/usr/bin/env python3
"""Benchmark of the hot path: GB/s of stream scanned (+ matches/sec) on
snort.dict, one process per GPU (BASELINE.json configs 3 and 4).

A "step" is one scan of the rank's whole stream shard (default 1 GiB of
seeded synthetic ASCII, generated on the device, resident in HBM before the
timed region) through the HIP kernel, writing the dense per-position match
ids (u32; the read_block contract).  Shards are independent streams (one per
rank, distinct seeds): weak scaling, no data-path collective.  The only
collective is the RCCL all-reduce of match counts and the max-over-ranks
time.  --layout split instead cuts ONE logical stream of N x --bytes into
rank shards (patternmatching_amd.shard.shard_plan: each rank generates its
shard plus the max_len-1 bytes before it as context), so the all-reduced
match count is that of the whole stream.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...

Prints one JSON line on rank 0.
"""
import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "GB/s stream scanned + matches/sec, snort.dict, 1/2/4/8 MI355X vs CPU ref"
DATA = os.path.join(REPO, "tests", "golden", "data")
DICTS = {"et": ["et.dict"], "snort": ["snort.dict"], "merged": ["snort.dict", "et.dict"]}
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md, HBM3E peak (spec)
WIDTH = {"dense": 4, "dense16": 2, "count": 0}  # bytes written per stream position


def parse():
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
                   help="ascii / bytes: seeded synthetic (DESIGN.md §5); ship: the reference's shipped "
                        "dictionaries_generated.stream tiled to --bytes (adversarial: deep matches)")
    p.add_argument("--seed", type=int, default=1)
    p.add_argument("--layout", default="shards", choices=["shards", "split"],
                   help="shards: an independent seeded stream per rank; split: one stream of N x --bytes "
                        "cut into rank shards with max_len-1 bytes of context (ascii / bytes streams)")
    p.add_argument("--cpu-sample", type=int, default=256 << 20, help="bytes of the CPU-baseline sample")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--score", action="store_true",
                   help="after timing, score the ids against the AC-DFA reliable instance on the device "
                        "(measure.c:174-190) and report FP/FN/partial rates (dense mode)")
    return p.parse_args()


def host_cores():
    """Host cores this job may use: the box exposes the whole machine to
    os.cpu_count() but gives a job a share (OMP_NUM_THREADS there)."""
    n = os.cpu_count() or 1
    share = os.environ.get("OMP_NUM_THREADS")
    if share and share.isdigit():
        n = min(n, int(share))
    return max(1, min(n, 16))


def cpu_baseline(args):
    """The reference's own per-byte AC loop (oracle/_ref/ref_driver, built from
    the reference's sources, mps_table[MPS_AC].read_char per byte): on 1 core
    over the first cpu_sample bytes of the stream, and on every host core as
    one process per core, each on its own seeded sample (the
    aggregate is the sum of the per-process rates).  Without that binary the
    C port of the loop (oracle/ac_oracle.c) is timed on 1 core.  Test
    infrastructure, used here only as the measured baseline."""
    mode = 0 if args.stream == "ascii" else 1
    paths = [os.path.join(DATA, d) for d in DICTS[args.dict]]
    ref = os.path.join(REPO, "oracle", "_ref", "ref_driver")
    sample = f"first {args.cpu_sample} bytes of the seed-{args.seed} {args.stream} stream, {args.dict}.dict"
    if os.path.exists(ref):
        try:
            r = subprocess.run([ref, "time", str(args.seed), str(mode), str(args.cpu_sample)] + paths,
                               check=True, capture_output=True, text=True, timeout=600)
            one = json.loads(r.stdout)
            single = {"value": round(one["MBps"] / 1000.0, 6), "unit": "GB/s", "cores": 1, "seconds": one["seconds"],
                      "nonnull": one["nonnull"], "sample": sample}
            P = host_cores()
            per = max(1 << 20, args.cpu_sample // 2)
            procs = [subprocess.Popen([ref, "time", str(args.seed + 1000 + k), str(mode), str(per)] + paths,
                                      stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True)
                     for k in range(P)]
            outs = [json.loads(p.communicate(timeout=900)[0]) for p in procs]
            agg = sum(o["MBps"] for o in outs) / 1000.0
            return {"value": round(agg, 6), "unit": "GB/s", "cores": P, "kind": "reference",
                    "sample": f"{P} concurrent processes (one per core), each the first {per} bytes of its own "
                              f"seeded {args.stream} stream (seeds {args.seed + 1000}..), {args.dict}.dict; "
                              "reference Core/src objects, mps_table[MPS_AC].read_char per byte; value = sum of "
                              "the per-process rates",
                    "per_core_min": round(min(o["MBps"] for o in outs) / 1000.0, 6),
                    "single_core": single}
        except (subprocess.SubprocessError, OSError, ValueError, KeyError):
            pass
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import patternmatching_amd as pm
    from oracle_lib import Oracle
    o = Oracle(paths)
    secs, nonnull = o.time_scan(pm.gen_stream(args.cpu_sample, args.seed, mode), threads=1)
    return {"value": round(args.cpu_sample / secs / 1e9, 6), "unit": "GB/s", "cores": 1, "kind": "port",
            "sample": sample + "; oracle/ac_oracle.c per-byte read_char", "seconds": secs, "nonnull": nonnull}


def load_traffic(workload_key):
    """HBM bytes per launch from the committed rocprofv3 PMC summary, if one
    exists for this exact workload (profiles/traffic.json)."""
    path = os.path.join(REPO, "profiles", "traffic.json")
    try:
        with open(path) as f:
            t = json.load(f).get(workload_key)
        return t
    except (OSError, ValueError):
        return None


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    # CPU leg first, before this process touches the GPU
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu and args.stream in ("ascii", "bytes"):
        cpu = cpu_baseline(args)

    import torch
    import torch.distributed as dist
    import patternmatching_amd as pm

    # one GPU per rank; a rehearsal with more ranks than GPUs (gloo) shares them
    dev = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev)
    # the RCCL path runs for world > 1; PM_BENCH_DIST=1 runs it at world 1 too
    # (one-GPU rehearsal of the multi-GPU code: init, barriers, all-reduces).
    # PM_BENCH_BACKEND=gloo rehearses several ranks on one GPU.
    use_dist = world > 1 or os.environ.get("PM_BENCH_DIST") == "1"
    backend = os.environ.get("PM_BENCH_BACKEND", "nccl")
    if use_dist:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)
    lib = pm.load()
    lib.pm_hip_set_device(dev)

    d = pm.Dictionary([os.path.join(DATA, x) for x in DICTS[args.dict]])
    m = pm.HipMatcher(args.kernel)
    m.add_dictionary(d)
    m.compile()

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
    if args.stream == "ship":
        import numpy as np
        ship = torch.from_numpy(np.fromfile(os.path.join(DATA, "dictionaries_generated.stream"), dtype=np.uint8))
        reps = (n + 64 + ship.numel() - 1) // ship.numel()
        text.copy_(ship.to("cuda").repeat(reps)[: n + 64])
    elif args.stream == "lines":
        m.gen_lines_device(text.data_ptr(), n + 64, seed, stream.cuda_stream)
    elif lib.pm_hip_gen_stream_device(text.data_ptr(), gen_off, pos0 + n + 64, seed,
                                      0 if args.stream == "ascii" else 1, stream.cuda_stream) != 0:
        raise RuntimeError(lib.pm_hip_last_error().decode())
    width = WIDTH[args.mode]
    out = torch.empty(n, dtype={4: torch.int32, 2: torch.int16}[width], device="cuda") if width else None
    count = torch.zeros(1, dtype=torch.int64, device="cuda")
    out_ptr = out.data_ptr() if out is not None else None

    def step():
        m.scan_device(text.data_ptr(), 0, pos0, n, out_ptr, count.data_ptr(), stream.cuda_stream, out_width=width or 4)

    # ac / auto pick their kernel by timing it (an RT launch, then two launches
    # of each DFA form): let that finish before the W warmups so the timed
    # steps run the held choice (pm_plugin.hip AUTO_HOLD)
    pick_launches = {"rt": 0, "ac": 5, "auto": 6}[args.kernel]
    for _ in range(pick_launches + args.warmup):
        step()
    torch.cuda.synchronize()
    if use_dist:
        dist.barrier()
    count.zero_()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        evs[k][0].record(stream)
        step()
        evs[k][1].record(stream)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if use_dist:
        dist.barrier()
    elapsed = t1 - t0
    kernel_ms = sum(a.elapsed_time(b) for a, b in evs) / args.steps

    stats = torch.tensor([elapsed, kernel_ms], dtype=torch.float64, device="cuda")
    matches = count.clone()
    if use_dist:
        dist.all_reduce(stats, op=dist.ReduceOp.MAX)
        dist.all_reduce(matches, op=dist.ReduceOp.SUM)  # RCCL over xGMI: the match-count reduction
    # after the timed region: all-matches (patterns ending at each position,
    # i.e. the suffix-chain length of each id) and, with --score, accuracy
    # against the reliable AC instance, both by pm_hip_score_device
    extra = {}
    if width == 4:
        sc = torch.zeros(5, dtype=torch.int64, device="cuda")
        m.score_device(out.data_ptr(), out.data_ptr(), n, sc.data_ptr(), stream.cuda_stream)
        allm = sc.clone()
        if args.score:
            ac = pm.HipMatcher("ac")
            ac.add_dictionary(d)
            ac.compile()
            ref = torch.empty(n, dtype=torch.int32, device="cuda")
            ac.scan_device(text.data_ptr(), 0, pos0, n, ref.data_ptr(), None, stream.cuda_stream)
            sc.zero_()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            m.score_device(out.data_ptr(), ref.data_ptr(), n, sc.data_ptr(), stream.cuda_stream)
            e1.record(stream)
            torch.cuda.synchronize()
            c = [int(v) for v in sc.tolist()]
            extra["accuracy"] = {"reliable": "AC-DFA (HIP)", "positions": n, "success": c[0],
                                 "false_pos_rate": c[3] / n, "false_neg_rate": c[2] / n, "partial_rate": c[1] / n,
                                 "score_ms": round(e0.elapsed_time(e1), 4)}
            del ref
            hist = torch.zeros(lib.pm_hip_n_patterns(m.obj) + 1, dtype=torch.int64, device="cuda")
            for _ in range(2):  # the second launch is timed (the first pays first-touch costs)
                hist.zero_()
                e0.record(stream)
                m.pattern_counts_device(out.data_ptr(), n, hist.data_ptr(), stream.cuda_stream)
                e1.record(stream)
                torch.cuda.synchronize()
            extra["pattern_counts"] = {"patterns_seen": int((hist > 0).sum().item()),
                                       "occurrences": int(hist.sum().item()),
                                       "ms": round(e0.elapsed_time(e1), 4)}
        if use_dist:
            dist.all_reduce(allm, op=dist.ReduceOp.SUM)
        extra["all_matches_per_step"] = int(allm[4].item())
    elapsed, kernel_ms = stats.tolist()
    total_matches = int(matches.item())

    # the same kernel's streaming floor, live on this GPU: variant 2 of
    # rt_scan_kernel runs the chunk loop's loads and stores with no lookups
    # (its ids are not matches; `out` is not used after this)
    floor = None
    if rank == 0 and args.kernel == "rt" and pos0 == 0:
        fts = []
        for r in range(4):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            rc = lib.pm_hip_debug_scan_variant(m.obj, 2, text.data_ptr(), n, out_ptr, width, None, stream.cuda_stream)
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
                     "what": "rt_scan_kernel variant 2 on this GPU: the same loads and stores, no lookups "
                             "(pm_hip_debug_scan_variant); kernel_over_floor = kernel_ms / floor kernel_ms"}

    if rank == 0:
        last_kernel = "RT" if m.kernel_last == 1 else {1: "AC dense rows", 2: "AC rows + records"}.get(m.dfa_form_last, "?")
        total_bytes = world * args.bytes * args.steps  # every rank scans --bytes positions
        value = total_bytes / elapsed / 1e9
        alg_per_pos = 1 + width  # 1 B read + the id written per position
        achieved = n * alg_per_pos / (kernel_ms * 1e-3) / 1e9
        workload_key = f"{args.dict}-{args.stream}-{n}-{args.mode}-{args.kernel}"
        tr = load_traffic(workload_key)
        traffic = tr["traffic_bytes"] if tr else None
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
                              "(splitmix64 per 1 KiB block), '\\n' after each, generated in HBM (DESIGN.md §5)"}.get(
                args.stream, "synthetic: seeded splitmix64 %s stream per GPU (DESIGN.md §5), generated in HBM; "
                             "dictionaries from the reference" % args.stream),
            "config": {
                "workload": f"{args.dict}.dict, {n} B {args.stream} stream per GPU, "
                            + {"dense": "dense u32 match id per position", "dense16": "dense u16 match id per position",
                               "count": "match count only"}[args.mode],
                "dict": args.dict,
                "stream_bytes_per_gpu": n,
                "mode": args.mode,
                "kernel": ("auto: RT, or after a deep RT launch (spill > 10%%) the fastest of RT and timed trials of "
                           "both AC-DFA forms (last launch: %s)" % last_kernel if args.kernel == "auto" else
                           "Aho-Corasick DFA, the faster of its two forms by timed trials (last launch: %s)" % last_kernel
                           if args.kernel == "ac" else "reverse-suffix-trie walk"),
                "pick_launches": pick_launches,
                "parallelism": (f"independent stream shards x{world}" if args.layout == "shards" else
                                f"one {world * args.bytes} B stream split x{world} (max_len-1 B context per shard)"),
                "layout": args.layout,
            },
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
            "cpu_baseline": cpu,
        }
        print(json.dumps(res), flush=True)
    if use_dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
