"""Multi-rank path on CPU (gloo, world_size 2): the shard plan is exact at
the seams and the all-reduced match count equals the single-process count.
The oracle stands in for the per-rank scan (no GPU here); the GPU-side seam
exactness is tests/test_gpu_parity.py::test_scan_device_shards_with_context."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import patternmatching_amd as pm
from patternmatching_amd.shard import scan_shard, shard_plan


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, result_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle_lib import DATA, Oracle
    o = Oracle([os.path.join(DATA, "snort.dict"), os.path.join(DATA, "et.dict")])
    ship = np.fromfile(os.path.join(DATA, "dictionaries_generated.stream"), dtype=np.uint8)
    text = np.concatenate([np.tile(ship, 8), pm.gen_stream(50_000, seed=4, mode=0)])

    def scan(part):
        o.reset()
        return o.scan_codes(part)

    sh = shard_plan(len(text), world, rank, o.max_len)
    mine = scan_shard(scan, text, sh)
    cnt = torch.tensor([int(np.count_nonzero(mine))], dtype=torch.int64)
    dist.all_reduce(cnt, op=dist.ReduceOp.SUM)
    parts = [None] * world
    dist.all_gather_object(parts, mine)
    if rank == 0:
        o.reset()
        whole = o.scan_codes(text)
        result_q.put((int(cnt.item()), int(np.count_nonzero(whole)), bool(np.array_equal(np.concatenate(parts), whole))))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_sharded_scan_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    total, single, exact = q.get(timeout=10)
    assert total == single
    assert exact


def test_shard_plan_covers_and_aligns():
    for n in (0, 1, 15, 16, 1000, 1 << 20):
        for world in (1, 2, 3, 8):
            prev = 0
            for r in range(world):
                sh = shard_plan(n, world, r, 347)
                assert sh.lo == prev and sh.lo <= sh.hi
                assert sh.lo % 16 == 0 or sh.lo == n
                assert sh.ctx_lo == max(0, sh.lo - 346)
                prev = sh.hi
            assert prev == n
