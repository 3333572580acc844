"""Partition 0 coded on the device (WEBP_AMD_P0=gpu; the default when the
rank's host-thread budget is below 8 threads, e.g. 8 ranks on a 16-CPU
quota): the host turns each frame's header (segment, filter and quantiser
headers, probability updates, skip probability: syntax_enc.c:187-245,
tree_enc.c:485-504) into fixed-probability tokens, k_p0_modes appends every
MB's segment id, skip flag and intra modes (tree_enc.c:313-347) from K3's
mbinfo, and K4 codes the stream beside the token partitions.

Parity: the same reference golden vectors as the host path (bit-exact
files), over the token loop (methods 3-6), VP8EncLoop (methods 0-2 with the
skip flag, token partitions, low_memory), segments with and without the
segment map, the autofilter, alpha and the partition-0 overflow re-run.
The engines are GpuBatch instances created under the setting (the
WebPEncode engine pool keeps engines across calls, so it is not used here)."""
import hashlib
import json
import os

import numpy as np
import pytest

from libwebp_amd.synth import syn_v1

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def sha(b):
    return hashlib.sha256(b).hexdigest()


@pytest.fixture
def p0dev(monkeypatch):
    monkeypatch.setenv("WEBP_AMD_P0", "gpu")


def _golden(name):
    return json.load(open(os.path.join(HERE, "golden", name)))


def test_p0_device_1080p_hbm_batch(gpu, kat, p0dev):
    import torch
    cases = [c for c in kat["survey"] if c["w"] == 1920]
    n = len(cases)
    buf = torch.empty(n * 1920 * 1080 * 4, dtype=torch.uint8, device="cuda")
    gpu.synth_device(buf.data_ptr(), 1920, 1080, 0, n)
    torch.cuda.synchronize()
    enc = gpu.GpuBatch(1920, 1080, n)
    enc.encode_device(buf.data_ptr(), n)
    for i, c in enumerate(cases):
        out = enc.output(i)
        assert len(out) == c["size"] and sha(out) == c["sha256"], i
    enc.close()


def test_p0_device_sweep(gpu, kat, p0dev):
    """The 80 random configurations (sizes 1..333, q 0..100, m3..m6,
    segments, sns, filter, sharpness, partition_limit)."""
    bad = []
    for c in kat["sweep"]:
        enc = gpu.GpuBatch(c["w"], c["h"], 1, **c["params"])
        enc.encode_host(syn_v1(c["w"], c["h"], c["frame"])[None])
        if sha(enc.output(0)) != c["sha256"]:
            bad.append((c["w"], c["h"], c["frame"], c["params"]))
        enc.close()
    assert not bad, bad


def test_p0_device_methods012_and_partitions(gpu, p0dev):
    """VP8EncLoop: the skip flag per MB (use_skip), token partitions,
    low_memory, the autofilter -- the reference's files."""
    from test_methods012 import CASES as M_CASES
    from test_partitions import CASES as P_CASES
    bad = []
    for cases, kat in ((M_CASES, _golden("methods012_kat.json")["cases"]),
                       (P_CASES, _golden("partitions_kat.json")["cases"])):
        for (w, h, f, kw), c in zip(cases, kat):
            enc = gpu.GpuBatch(w, h, 1, **kw)
            enc.encode_host(syn_v1(w, h, f)[None])
            out = enc.output(0)
            enc.close()
            if (len(out), sha(out)) != (c["size"], c["sha256"]):
                bad.append((w, h, f, kw))
    assert not bad, bad


def test_p0_device_batch_matches_host(gpu, monkeypatch):
    """Same batch, both placements: identical files (segment maps, intra-4
    contexts across MB rows, odd sizes)."""
    import torch
    w, h, n = 333, 257, 6
    frames = np.stack([syn_v1(w, h, f) for f in range(n)])
    buf = torch.from_numpy(frames).to("cuda:0")
    torch.cuda.synchronize()
    for kw in ({"quality": 75.0, "method": 4}, {"quality": 40.0, "method": 6, "segments": 4},
               {"quality": 90.0, "method": 3, "segments": 1}, {"quality": 65.0, "method": 0}):
        out = {}
        for mode in ("host", "gpu"):
            monkeypatch.setenv("WEBP_AMD_P0", mode)
            enc = gpu.GpuBatch(w, h, n, **kw)
            enc.encode_device(buf.data_ptr(), n)
            out[mode] = [enc.output(f) for f in range(n)]
            enc.close()
        assert out["host"] == out["gpu"], kw


def test_p0_device_overflow_rerun(gpu, kat, p0dev):
    """The partition-0 overflow retry (frame_enc.c:869-876) with partition 0
    on the device: 5120x5120 q95 m4, 3 passes, the reference's file."""
    import torch
    (c,) = kat["p0_overflow"]
    w, h = c["w"], c["h"]
    buf = torch.empty(w * h * 4, dtype=torch.uint8, device="cuda")
    gpu.synth_device(buf.data_ptr(), w, h, c["frame"], 1)
    torch.cuda.synchronize()
    enc = gpu.GpuBatch(w, h, 1, **c["params"])
    enc.encode_device(buf.data_ptr(), 1)
    out, err = enc.output(0), enc.error(0)
    enc.close()
    assert err == 0
    assert len(out) == c["size"] and sha(out) == c["sha256"]


def test_p0_device_alpha(gpu, p0dev, monkeypatch):
    """VP8X + ALPH + VP8 with the device partition 0: the same file as the host's."""
    img = syn_v1(48, 40, 2).copy()
    img[::3, ::5, 3] = 100
    outs = []
    for mode in ("gpu", "host"):
        monkeypatch.setenv("WEBP_AMD_P0", mode)
        enc = gpu.GpuBatch(48, 40, 1, alpha_quality=80)
        enc.encode_host(img[None])
        assert enc.error(0) == 0
        outs.append(enc.output(0))
        enc.close()
    assert outs[0][12:16] == b"VP8X" and outs[0] == outs[1]
