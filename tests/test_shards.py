"""BASELINE.json configs[2] (2048 x 1080p, q75 m4, 8 ranks of 256 frames)
on the one GPU a test box has.

* every rank's shard: frames [256 r, 256 r + 256) for r = 0..7 are generated
  in HBM and encoded as one 256-frame batch each -- exactly the batch a rank
  of `bench.py --gpus 8` encodes -- and every frame that
  tests/golden/shard_kat.json pins (31 frames up to f2047, reference libwebp
  SHA-256s made by tests/golden/make_shard_golden.py) must match;
* the rank path itself with the real encoder: `bench.py --gpus 2` as two
  processes on device 0 over gloo (the test-only backend; RCCL between two
  ranks of one GPU is not what the driver's 8-GPU run exercises anyway),
  checking the timed batch of both ranks against the same known answers;
* host-thread placement: the engines' CPU share lies on the GPU's NUMA node.
"""
import hashlib
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
W, H, B, RANKS = 1920, 1080, 256, 8


def shard_kat():
    with open(os.path.join(ROOT, "tests", "golden", "shard_kat.json")) as fh:
        k = json.load(fh)
    assert (k["width"], k["height"], k["quality"], k["method"]) == (W, H, 75.0, 4)
    return {int(f): v for f, v in k["frames"].items()}


def test_shard_kat_covers_every_rank():
    """CPU: the known answers pin the first, a middle and the last frame of
    each of the 8 ranks' shards"""
    frames = shard_kat()
    for r in range(RANKS):
        mine = [f for f in frames if r * B <= f < (r + 1) * B]
        assert r * B in mine and (r + 1) * B - 1 in mine and len(mine) >= 3, r


@pytest.mark.gpu
def test_every_rank_shard_on_one_gpu(gpu):
    import torch
    frames = shard_kat()
    fs = 4 * W * H
    buf = torch.empty(B * fs, dtype=torch.uint8, device="cuda:0")
    enc = gpu.GpuBatch(W, H, B, quality=75.0, method=4)
    checked = 0
    for r in range(RANKS):
        first = r * B
        gpu.synth_device(buf.data_ptr(), W, H, first, B)
        torch.cuda.synchronize()
        enc.encode_device(buf.data_ptr(), B)
        for f, want in sorted(frames.items()):
            if not first <= f < first + B:
                continue
            src = buf[(f - first) * fs:(f - first + 1) * fs].cpu().numpy().tobytes()
            assert hashlib.sha256(src).hexdigest()[:16] == want["in_sha"], f
            out = enc.output(f - first)
            assert len(out) == want["size"], (f, len(out))
            assert hashlib.sha256(out).hexdigest() == want["sha256"], f
            checked += 1
        assert all(enc.error(i) == 0 for i in range(B)), r
    enc.close()
    assert checked == len(frames) == 31


@pytest.mark.gpu
def test_two_real_ranks_on_one_gpu(gpu):
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR",
              "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--dist-backend", "gloo", "--same-device", "--engines", "1",
                        "--steps", "1", "--warmup", "1", "--no-cpu", "--no-host-input"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["config"]["frames_per_gpu"] == B
    # frames 0..7, 131, 255 (rank 0) and 256, 387, 511 (rank 1)
    assert line["kat_check"].startswith("ok: 13 timed-batch frames on 2 rank(s)"), line
    assert line["value"] > 0


@pytest.mark.gpu
def test_rccl_rank_path_one_gpu(gpu):
    """configs[2]'s collective over RCCL itself: bench.py as one rank with its
    process group created on the nccl backend (RCCL on ROCm) -- the real
    encoder's timed batch, the all-gather of the encoded sizes and the max /
    sum reductions of the timing and the known-answer counts all go through
    RCCL on the GPU (two ranks cannot share one GPU under RCCL; the 8-GPU
    run is the driver's)"""
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR",
              "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--force-pg",
                        "--dist-backend", "nccl", "--engines", "1", "--steps", "1",
                        "--warmup", "0", "--no-cpu", "--no-other-input", "--input", "hbm"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["collectives"].startswith("nccl, 1 rank(s)"), line
    assert line["kat_check"].startswith("ok: 10 timed-batch frames on 1 rank(s)"), line
    assert line["output_bytes_per_frame"] > 0


@pytest.mark.gpu
def test_host_cpus_on_numa_node(gpu):
    """the engines' CPU share: inside this process's affinity and on the GPU's
    NUMA node when sysfs names one (else unpinned)"""
    cpus = gpu.host_cpus(0)
    allowed = os.sched_getaffinity(0)
    assert set(cpus) <= allowed
    if cpus:
        assert len(cpus) == len(set(cpus))
