"""Multi-rank path of bench.py on CPU (gloo, world_size 2): frame sharding,
the encoded-size all-gather and the max-over-ranks timing."""
import os
import socket
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    import bench
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    first, n = bench.shard(rank, 4)
    sizes = torch.arange(first, first + n, dtype=torch.int64) * 10 + 1
    allsizes = bench.gather_sizes(sizes, world)
    t = bench.max_over_ranks(1.0 + rank, world, torch.device("cpu"))
    q.put((rank, [s.tolist() for s in allsizes], t))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_two_ranks():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    expect = [[1, 11, 21, 31], [41, 51, 61, 71]]
    for rank, allsizes, t in res:
        assert allsizes == expect          # disjoint shards, frames 0..7
        assert t == 2.0                    # max over ranks


def test_shard_disjoint():
    import bench
    seen = set()
    for r in range(8):
        first, n = bench.shard(r, 256)
        fr = set(range(first, first + n))
        assert not (fr & seen)
        seen |= fr
    assert seen == set(range(2048))
