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


def test_launcher_two_ranks_stub():
    """`bench.py --gpus 2` outside torchrun starts torch.distributed.run with
    two ranks itself; with the CPU test double (gloo) the full rank path runs:
    sharding, warm-up, timed loop, size all-gather, max-over-ranks timing and
    the timed-batch known-answer check summed over the ranks."""
    import json
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--stub", "--gpus", "2",
                        "--steps", "2", "--warmup", "1"], capture_output=True, text=True,
                       timeout=240, env=env, cwd="/tmp")
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["steps"] == 2 and line["scaling"] == "weak"
    # frames 0..7, 131, 255 (rank 0) and 256, 387, 511 (rank 1) are pinned
    assert line["kat_check"].startswith("ok: 13 timed-batch frames on 2 rank(s)")
    # the stub's sizes are 100 + f % 7 bytes for frames 0..511
    assert line["output_bytes_per_frame"] == round(sum(100 + f % 7 for f in range(512)) / 512, 1)
