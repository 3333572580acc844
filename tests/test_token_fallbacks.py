"""The token rows' regrow (host/gpu_batch.c k3_settle), run on purpose:
WEBP_AMD_TEST_TINY_TOKENS=1 starts an engine with token rows of 64 tokens,
so in its first K3 launch every MB row runs out of room (K3 stops writing
the row and reports VP8G_ERR_ARENA, counting the row's tokens on); the host
reads the rows' counts, widens the rows to hold the longest, keeps the rows
of the frames the launch skipped (a partition-0 re-run's final frames) and
runs the launch again from the saved pass state (d_rerun_snap). The
bitstreams must equal the reference's known answers: the m4 survey KATs (K3
and K3X), an m6 sweep case (trellis kernel) and multi-pass size / PSNR
searches (pass state restored before the re-run, the token-cost estimate
read from the rows)."""
import hashlib
import json
import os

import numpy as np
import pytest

from libwebp_amd.synth import syn_v1

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def sha(b):
    return hashlib.sha256(b).hexdigest()


@pytest.fixture
def tiny(monkeypatch, gpu):
    monkeypatch.setenv("WEBP_AMD_TEST_TINY_TOKENS", "1")
    return gpu


def test_survey_512_batch_tiny_tokens(tiny, kat):
    cases = [c for c in kat["survey"] if c["w"] == 512]
    frames = np.stack([syn_v1(512, 512, c["frame"]) for c in cases])
    enc = tiny.GpuBatch(512, 512, len(cases))   # few frames: K3X
    enc.encode_host(frames)
    for i, c in enumerate(cases):
        assert sha(enc.output(i)) == c["sha256"], c["frame"]
    enc.encode_host(frames)                      # second call: the grown buffers
    for i, c in enumerate(cases):
        assert sha(enc.output(i)) == c["sha256"], c["frame"]
    enc.close()


def test_survey_1080p_batch_tiny_tokens(tiny, kat):
    import torch
    cases = [c for c in kat["survey"] if c["w"] == 1920]
    n = len(cases)
    buf = torch.empty(n * 1920 * 1080 * 4, dtype=torch.uint8, device="cuda")
    tiny.synth_device(buf.data_ptr(), 1920, 1080, 0, n)
    torch.cuda.synchronize()
    enc = tiny.GpuBatch(1920, 1080, n)
    enc.encode_device(buf.data_ptr(), n)
    for i, c in enumerate(cases):
        assert sha(enc.output(i)) == c["sha256"], i
    enc.close()


def test_one_frame_per_workgroup_kernel_tiny_tokens(tiny, kat):
    """More frames than K3X splits (one workgroup per frame): the 1080p KATs
    repeated past VP8G_XSPLIT_MAX_FRAMES."""
    import torch
    cases = [c for c in kat["survey"] if c["w"] == 1920]
    n = 72
    buf = torch.empty(n * 1920 * 1080 * 4, dtype=torch.uint8, device="cuda")
    for k in range(0, n, len(cases)):
        tiny.synth_device(buf[k * 1920 * 1080 * 4:].data_ptr(), 1920, 1080, 0,
                          min(len(cases), n - k))
    torch.cuda.synchronize()
    enc = tiny.GpuBatch(1920, 1080, n)
    enc.encode_device(buf.data_ptr(), n)
    for i in range(n):
        assert sha(enc.output(i)) == cases[i % len(cases)]["sha256"], i
    enc.close()


def test_trellis_sweep_case_tiny_tokens(tiny, kat):
    cases = [c for c in kat["sweep"] if c["params"]["method"] == 6 and c["w"] * c["h"] > 20000]
    assert cases
    for c in cases[:3]:
        enc = tiny.GpuBatch(c["w"], c["h"], 1, **c["params"])
        enc.encode_host(syn_v1(c["w"], c["h"], c["frame"])[None])
        out = enc.output(0)
        enc.close()
        assert sha(out) == c["sha256"], c


def test_multipass_tiny_tokens(tiny):
    k = json.load(open(os.path.join(ROOT, "tests", "golden", "multipass_kat.json")))["cases"]
    picked = [c for c in k if c["params"].get("target_size") or c["params"].get("target_PSNR")]
    for c in picked[:4]:
        enc = tiny.GpuBatch(c["w"], c["h"], 1, **c["params"])
        enc.encode_host(syn_v1(c["w"], c["h"], c["frame"])[None])
        out = enc.output(0)
        assert enc.error(0) == 0
        enc.close()
        assert (len(out), sha(out)) == (c["size"], c["sha256"]), c["params"]
