"""Dithered RGB -> YUV import (config->preprocessing & 2, cwebp -pre 2):
WebPEncode of an ARGB picture converts with WebPPictureARGBToYUVADithered
(src/enc/webp_enc.c:357-365), whose rounding terms come from the VP8Random
generator (src/utils/random_utils.{h,c}; picture_csp_enc.c:150-166,520-619).

Parity: bit-exact bitstreams. Golden vectors from the reference build
(tests/golden/dither_kat.json, make_options_golden.py); the oracle's
restatement is checked against them on CPU, the GPU path (host-generated
rounding terms fed to K1) through WebPEncode and the batch API.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from libwebp_amd.synth import syn_v1

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CASES = [
    (64, 48, 0, {"quality": 75.0, "method": 4, "preprocessing": 2, "use_argb": True}),
    (33, 17, 1, {"quality": 20.0, "method": 4, "preprocessing": 2, "use_argb": True}),
    (333, 257, 2, {"quality": 90.0, "method": 6, "preprocessing": 3, "use_argb": True}),
    (128, 97, 3, {"quality": 50.0, "method": 2, "preprocessing": 2, "use_argb": True}),
    (512, 512, 0, {"quality": 75.0, "method": 4, "preprocessing": 2, "use_argb": True}),
    (1, 1, 4, {"quality": 0.0, "method": 4, "preprocessing": 2, "use_argb": True}),
]


def kat():
    return json.load(open(os.path.join(ROOT, "tests", "golden", "dither_kat.json")))["cases"]


def sha(b):
    return hashlib.sha256(b).hexdigest()


def test_golden_inputs_pinned():
    k = kat()
    assert len(k) == len(CASES)
    for (w, h, f, kw), c in zip(CASES, k):
        assert (c["w"], c["h"], c["frame"], c["params"]) == (w, h, f, kw)
        assert sha(syn_v1(w, h, f).tobytes())[:16] == c["in_sha"]


@pytest.mark.parametrize("i", range(len(CASES)))
def test_oracle_matches_reference(i):
    from oracle import oracle
    w, h, f, kw = CASES[i]
    kw = {k: v for k, v in kw.items() if k != "use_argb"}
    assert sha(oracle.encode_rgba(syn_v1(w, h, f), **kw)) == kat()[i]["sha256"]


@pytest.mark.gpu
def test_gpu_webpencode_dither(gpu):
    for (w, h, f, kw), c in zip(CASES, kat()):
        out = gpu.encode_rgba(syn_v1(w, h, f), **kw)
        assert (len(out), sha(out)) == (c["size"], c["sha256"]), (w, h, f, kw)


@pytest.mark.gpu
def test_gpu_batch_dither(gpu):
    """The batch API dithers like cwebp -pre 2 (which imports to ARGB)."""
    import torch
    w, h, n = 333, 257, 3
    k = kat()
    frames = np.stack([syn_v1(w, h, 2) for _ in range(n)])
    kw = {k_: v for k_, v in CASES[2][3].items() if k_ != "use_argb"}
    enc = gpu.GpuBatch(w, h, n, **kw)
    buf = torch.from_numpy(frames).to("cuda:0")
    torch.cuda.synchronize()
    enc.encode_device(buf.data_ptr(), n)
    for f in range(n):
        assert sha(enc.output(f)) == k[2]["sha256"], f
    enc.close()
