"""bench.py keeps the driver's contract: one JSON line with the required
keys, whole-job value = bytes / wall time, roofline from the kernel time,
and the CPU baseline leg (the reference's loop; the C port without it)."""
import argparse
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REQUIRED = ["metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"]


def _bench_args(**kw):
    sys.path.insert(0, REPO)
    import bench
    a = dict(gpus=1, steps=1, warmup=0, dict="et", bytes=1 << 20, mode="dense", kernel="rt", stream="ascii", seed=1,
             cpu_sample=1 << 20, cpu_cores=2, no_cpu=False, no_extra=False, score=False, layout="shards")
    a.update(kw)
    return bench, argparse.Namespace(**a)


def test_cpu_baseline_leg_small_sample():
    """The CPU leg runs without a GPU: the reference's loop on a 1 MiB
    sample (one process per host core) or, without that binary, the port."""
    bench, args = _bench_args()
    cpu = bench.cpu_baseline(args)
    assert cpu["unit"] == "GB/s" and cpu["value"] > 0 and cpu["cores"] >= 1
    assert cpu["kind"] in ("reference", "port")
    assert cpu["port"]["value"] > 0 and cpu["port"]["cores"] == 1  # the C port's rate, always stated
    assert cpu["nproc"] >= cpu["share"] >= 1
    if cpu["kind"] == "reference":
        assert cpu["single_core"]["nonnull"] == cpu["port"]["nonnull"]  # same bytes, same matches
        assert cpu["per_core_min"] > 0 and cpu["cores"] == 2


def test_hbm_peak_is_the_librarys():
    bench, _ = _bench_args()
    import patternmatching_amd as pm
    assert pm.load().pm_hip_hbm_peak_gbs() == bench.HBM_PEAK_GBS == 8000.0


def test_cpu_baseline_lines_sample():
    """The deep leg's sample: a lines stream of the dictionary, generated on
    the host (no device), timed through the reference loop and the port."""
    bench, args = _bench_args()
    cpu = bench.cpu_baseline(args, stream="lines", sample_bytes=1 << 20, multi=False)
    assert cpu["value"] > 0 and cpu["cores"] == 1 and "lines" in cpu["sample"]
    if cpu["kind"] == "reference":
        assert cpu["single_core"]["nonnull"] == cpu["port"]["nonnull"] > 0.9 * (1 << 20)


def _rehearse(extra, env=None):
    cmd = [sys.executable, os.path.join(REPO, "bench.py")] + extra
    e = dict(os.environ, PM_BENCH_REHEARSE="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=e, cwd=REPO)


def test_gpus_flag_starts_that_many_ranks_without_a_launcher():
    """`bench.py --gpus 2` with no WORLD_SIZE starts two ranks itself (the
    rendezvous + collectives rehearsed on gloo without a GPU); the CPU leg
    runs first and reaches rank 0's line at N = 2."""
    r = _rehearse(["--gpus", "2", "--dict", "et", "--cpu-sample", str(1 << 20), "--cpu-cores", "2",
                   "--no-extra"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["rehearsal"] and d["n_gpus"] == 2 and d["world_size"] == 2
    assert d["rank_sum"] == 3.0 and sorted(x["rank"] for x in d["per_rank"]) == [0, 1]
    assert len({x["pid"] for x in d["per_rank"]}) == 2
    assert d["cpu_baseline"]["value"] > 0


def test_eight_rank_rehearsal_shares_one_compile(tmp_path):
    """The driver's 8-GPU run, rehearsed on the CPU: `bench.py --gpus 8`
    starts eight ranks (gloo), and the start-up protocol runs for real on the
    host -- rank 0 flattens the automaton into the image cache, ranks 1-7
    read it after the barrier instead of compiling (measure.c:324-332's
    loop is what the ranks then shard).  Every rank reports its start-up."""
    cache = tmp_path / "imgcache"
    r = _rehearse(["--gpus", "8", "--dict", "et", "--no-cpu", "--no-extra", "--image-cache", str(cache)])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["rehearsal"] and d["n_gpus"] == 8 and d["world_size"] == 8
    assert d["rank_sum"] == 36.0 and sorted(x["rank"] for x in d["per_rank"]) == list(range(8))
    assert len({x["pid"] for x in d["per_rank"]}) == 8
    su = {x["rank"]: x["startup"] for x in d["per_rank"]}
    assert su[0]["image_cache"] == "miss"
    assert all(su[k]["image_cache"] == "hit" for k in range(1, 8)), su
    assert all(su[k]["compile_ms"] > 0 and su[k]["dict_load_ms"] > 0 for k in range(8))
    assert any(p.name.endswith(".img") for p in cache.iterdir())


def test_world_size_mismatch_is_an_error():
    r = _rehearse(["--gpus", "4", "--no-cpu"], env={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr


def test_more_ranks_than_gpus_is_refused_under_rccl():
    """Under RCCL a rank per GPU: a node world larger than the visible GPUs
    exits 3 with a message before any collective (instead of two ranks
    sharing a GPU and hanging in one); no rendezvous is attempted."""
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--no-cpu"]
    e = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", LOCAL_WORLD_SIZE="4096",
             MASTER_ADDR="127.0.0.1", MASTER_PORT="1")
    for k in ("PM_BENCH_REHEARSE", "PM_BENCH_BACKEND"):
        e.pop(k, None)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=e, cwd=REPO)
    assert r.returncode == 3, (r.returncode, r.stderr[-2000:])
    assert "one GPU per rank" in r.stderr


def _run(extra, env=None):
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--bytes", str(16 << 20), "--steps", "2", "--warmup", "1",
           "--no-cpu"] + extra
    e = dict(os.environ)
    e.update(env or {})
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=e, cwd=REPO)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


@pytest.mark.gpu
def test_bench_json_line_contract():
    d = _run([])
    for k in REQUIRED:
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["warmup"] == 1 and d["higher_is_better"] is True
    assert d["scaling"] == "weak" and d["unit"] == "GB/s" and d["dtype"] == "u8" and d["vs_baseline"] is None
    assert "workload" in d["config"]
    su = d["per_rank"][0]["startup"]  # start-up per rank
    assert su["compile_ms"] > 0 and su["upload_ms"] >= 0 and su["image_bytes"] > 0 and su["image_cache"] == "off"
    assert su["runtime_init_ms"] >= 0 and su["dict_load_ms"] > 0
    r = d["roofline"]
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == 8000.0
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    # achieved = 5 algorithmic B per position / kernel time; value = bytes / wall time
    assert abs(r["achieved"] - (16 << 20) * 5 / (d["kernel_ms"] * 1e-3) / 1e9) / r["achieved"] < 0.01
    assert abs(d["value"] - (16 << 20) / (d["ms_per_step"] * 1e-3) / 1e9) / d["value"] < 0.02
    assert d["matches_per_step"] > 0.8 * (16 << 20)  # snort on ASCII: ~92 % non-null


@pytest.mark.gpu
def test_bench_rccl_path_at_world_one():
    """PM_BENCH_DIST=1: the multi-GPU code (RCCL init, barriers, the max and
    sum all-reduces) at world size 1 gives the same match count."""
    plain = _run(["--mode", "count"])
    env = {"PM_BENCH_DIST": "1", "RANK": "0", "LOCAL_RANK": "0", "WORLD_SIZE": "1", "MASTER_ADDR": "127.0.0.1",
           "MASTER_PORT": "29533", "HSA_ENABLE_IPC_MODE_LEGACY": "0"}
    dist = _run(["--mode", "count"], env)
    assert dist["matches_per_step"] == plain["matches_per_step"]
    assert dist["n_gpus"] == 1


@pytest.mark.gpu
def test_bench_shipped_stream_and_score():
    """--stream ship (deep matches everywhere) with --score: the RT ids equal
    the AC instance's at every position."""
    d = _run(["--stream", "ship", "--score", "--dict", "et"])
    acc = d["accuracy"]
    assert acc["success"] == acc["positions"] == 16 << 20
    assert acc["false_pos_rate"] == acc["false_neg_rate"] == acc["partial_rate"] == 0.0
    assert d["cpu_baseline"] is None


@pytest.mark.gpu
def test_bench_split_layout_two_ranks_match_one_stream():
    """--layout split with 2 ranks (gloo rehearsal: both ranks on this GPU)
    cuts one 32 MiB stream into shards with max_len-1 bytes of context; the
    all-reduced match count equals one rank scanning the whole stream."""
    whole = _run(["--mode", "count", "--bytes", str(32 << 20)])
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29541", os.path.join(REPO, "bench.py"),
           "--gpus", "2", "--bytes", str(16 << 20), "--steps", "2", "--warmup", "1", "--no-cpu", "--mode", "count",
           "--layout", "split"]
    e = dict(os.environ, PM_BENCH_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=e, cwd=REPO)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    two = json.loads(lines[0])
    assert two["n_gpus"] == 2 and two["config"]["layout"] == "split"
    assert two["matches_per_step"] == whole["matches_per_step"]


@pytest.mark.gpu
def test_bench_gpus_two_self_launched_sums_two_single_runs():
    """`bench.py --gpus 2` with no launcher on a one-GPU box (two ranks share
    it; gloo rehearsal backend): n_gpus 2, per-rank rates, and the reduced
    count equals single-rank runs of the two shards (seeds 1 and 2)."""
    one = _run(["--mode", "count", "--no-extra"])
    two_seed = _run(["--mode", "count", "--no-extra", "--seed", "2"])
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--bytes", str(16 << 20), "--steps", "2",
           "--warmup", "1", "--no-cpu", "--mode", "count", "--no-extra"]
    e = dict(os.environ, PM_BENCH_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        e.pop(k, None)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=e, cwd=REPO)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["world_size"] == 2 and len(d["per_rank"]) == 2
    assert d["matches_per_step"] == one["matches_per_step"] + two_seed["matches_per_step"]
    assert d["rank_spread"] >= 1.0


@pytest.mark.gpu
def test_bench_default_extras():
    """The default run's count_only and deep objects (small sizes): the deep
    lines stream through the auto kind picks a DFA form, count-only counts
    the same matches as the dense run."""
    d = _run([])
    c = d["count_only"]
    assert c["matches_per_step"] == d["matches_per_step"] and c["roofline"]["frac"] > 0
    deep = d["deep"]
    assert deep["stream"] == "lines" and deep["kernel_ms"] > 0 and deep["picked"] in (
        "RT", "AC dense rows", "AC rows + records", "AC rows + records (16-B record loads)",
        "AC rows + records (64-B deep blocks)", "AC rows + records (two chains per lane)")
    assert deep["matches_per_step"] > 0.5 * (16 << 20)
    # the DFA legs' own bound, measured live over the object's table (the
    # achieved side needs a PMC entry for this exact workload: none here)
    g = deep["gather_roofline"]
    assert g["bound"] == "gathers" and g["ceiling"] > 1.0 and g["ceiling_loads"] > 0
