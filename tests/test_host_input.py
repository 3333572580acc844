"""The host-input path (WebPGpuBatchEncodeRGBAHost, bench.py's `value`) from
page-locked memory: the upload goes to an SDMA engine (host/h2d_sdma.c), the
streams stay bit-exact with the reference's known answers, including a batch
whose frames sit at a padded stride and a second call on the same engine."""
import hashlib

import numpy as np
import pytest

from libwebp_amd.synth import syn_v1

pytestmark = pytest.mark.gpu


def sha(b):
    return hashlib.sha256(b).hexdigest()


def pinned_frames(frames, pad=0):
    import torch
    n, h, w = frames.shape[:3]
    fs = h * w * 4 + pad
    buf = torch.zeros(n * fs, dtype=torch.uint8, pin_memory=True)
    for i in range(n):
        buf[i * fs:i * fs + h * w * 4] = torch.from_numpy(frames[i].reshape(-1))
    assert buf.is_pinned()
    return buf, fs


@pytest.mark.parametrize("pad", [0, 4096 + 64])
def test_pinned_upload_matches_kat(gpu, kat, pad):
    cases = [c for c in kat["survey"] if c["w"] == 512]
    frames = np.stack([syn_v1(512, 512, c["frame"]) for c in cases])
    buf, fs = pinned_frames(frames, pad)
    enc = gpu.GpuBatch(512, 512, len(cases))
    for _ in range(2):   # the second call reuses the engine's device buffer
        enc.encode_host_ptr(buf.data_ptr(), len(cases), frame_stride=fs)
        for i, c in enumerate(cases):
            out = enc.output(i)
            assert len(out) == c["size"] and sha(out) == c["sha256"], (pad, c["frame"])
    enc.close()
