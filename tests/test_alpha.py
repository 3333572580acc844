"""Lossy pictures with alpha: VP8X + ALPH + VP8 (src/enc/syntax_enc.c:149-185,
src/enc/alpha_enc.c).

Parity: the 'VP8 ' chunk is byte-identical to the reference encoder's (the
alpha-weighted chroma import, picture_csp_enc.c:388-424, and the transparent
area cleanup, picture_tools_enc.c:99-168, both feed it), and the ALPH chunk
decodes to exactly the input alpha plane (alpha_quality 100 = lossless). The
ALPH bytes themselves come from our VP8L engine (ALPH mode, see
oracle/vp8l_model.py) and are not the reference's. Golden vectors:
tests/golden/alpha_kat.json (make_alpha_golden.py, reference build).
"""
import hashlib
import json
import os

import numpy as np
import pytest

from libwebp_amd.synth import syn_v1
from oracle import vp8l_model as M

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def alpha_frame(w, h, f):
    """syn-v1 RGB with an alpha plane: ramps, a fully transparent block,
    partial-alpha noise, an opaque band (every cleanup/import case)."""
    img = syn_v1(w, h, f)
    yy, xx = np.mgrid[0:h, 0:w]
    a = ((xx * 5 + yy * 3 + 31 * f) % 320).clip(0, 255).astype(np.uint8)
    a[h // 4: h // 4 + 24, w // 5: w // 5 + 40] = 0
    rng = np.random.default_rng(100 + f)
    a[h // 2:, : w // 3] = rng.integers(0, 256, size=a[h // 2:, : w // 3].shape, dtype=np.uint8)
    a[-9:, :] = 255
    img[..., 3] = a
    return img


def logo_frame(w, h, f):
    """syn-v1 RGB with a logo-like alpha plane of three levels: an opaque
    disc, a transparent background, half-transparent diagonal blocks (the
    reference codes such planes with a palette)."""
    img = syn_v1(w, h, f)
    yy, xx = np.mgrid[0:h, 0:w]
    a = np.zeros((h, w), np.uint8)
    a[(xx - w / 2) ** 2 + (yy - h / 2) ** 2 < (min(w, h) / 3) ** 2] = 255
    a[(xx // 8 + yy // 8 + f) % 5 == 0] = 128
    img[..., 3] = a
    return img


def kat():
    return json.load(open(os.path.join(ROOT, "tests", "golden", "alpha_kat.json")))


def chunks(data):
    return dict(M.riff_chunks(data))


def test_golden_vectors_self_consistent():
    k = kat()
    assert k["cases"]
    for c in k["cases"]:
        img = alpha_frame(c["w"], c["h"], c["frame"])
        assert hashlib.sha256(img.tobytes()).hexdigest()[:16] == c["in_sha"]




def check(data, img, case):
    ch = chunks(data)
    assert [t for t, _ in M.riff_chunks(data)] == [b"VP8X", b"ALPH", b"VP8 "]
    assert hashlib.sha256(ch[b"VP8 "]).hexdigest() == case["vp8_sha256"]
    # decoded with the own decoder (oracle/webp_dec.c, pinned against the
    # reference decoder in tests/test_decoder.py)
    from oracle import oracle
    dec = oracle.decode_rgba(data)
    if case["alpha_quality"] < 100:   # the reference's level-reduced plane
        assert hashlib.sha256(dec[..., 3].tobytes()).hexdigest() == case["alpha_sha256"]
        assert chunks(data)[b"ALPH"][0] >> 4 == 1   # ALPHA_PREPROCESSED_LEVELS
    else:
        assert np.array_equal(dec[..., 3], img[..., 3])
    assert hashlib.sha256(dec[..., :3].tobytes()).hexdigest() == case["rgb_sha256"]


@pytest.mark.gpu
def test_gpu_batch_alpha_frames(gpu):
    import torch
    for case in kat()["cases"]:
        if case["api"] != "batch":
            continue
        w, h, f = case["w"], case["h"], case["frame"]
        frames = np.stack([alpha_frame(w, h, f), syn_v1(w, h, f + 1)])
        enc = gpu.GpuBatch(w, h, 2, quality=case["q"], method=case["m"], exact=case["exact"],
                           alpha_compression=case["alpha_compression"],
                           alpha_quality=case["alpha_quality"])
        buf = torch.from_numpy(frames).to("cuda:0")
        torch.cuda.synchronize()
        enc.encode_device(buf.data_ptr(), 2)
        check(enc.output(0), frames[0], case)
        assert chunks(enc.output(1)).keys() == {b"VP8 "}   # opaque frame: no VP8X/ALPH
        if case["alpha_compression"] == 0:
            assert chunks(enc.output(0))[b"ALPH"][0] & 3 == 0   # ALPHA_NO_COMPRESSION
        enc.close()


@pytest.mark.gpu
def test_gpu_api_alpha(gpu):
    for case in kat()["cases"]:
        if case["api"] != "webpencode":
            continue
        img = alpha_frame(case["w"], case["h"], case["frame"])
        data = gpu.encode_rgba(img, quality=case["q"], method=case["m"], exact=case["exact"],
                               alpha_compression=case["alpha_compression"],
                               alpha_quality=case["alpha_quality"])
        check(data, img, case)


@pytest.mark.gpu
@pytest.mark.parametrize("kind,w,h,f,m", [("logo", 512, 384, 0, 4), ("frame", 200, 130, 3, 4),
                                          ("logo", 97, 61, 2, 6), ("frame", 333, 257, 5, 2)])
def test_gpu_alph_matches_model(gpu, kind, w, h, f, m):
    """the ALPH payload (VP8L engine in ALPH mode, its entropy mode / palette
    chosen per frame) equals the model's alpha-plane stream"""
    img = (logo_frame if kind == "logo" else alpha_frame)(w, h, f)
    data = gpu.encode_rgba(img, quality=75.0, method=m, exact=1)
    alph = chunks(data)[b"ALPH"]
    assert alph[0] & 3 == 1
    assert alph[1:] == M.encode(img[..., 3], method=m, alpha_plane=True)


@pytest.mark.gpu
def test_gpu_alph_effort_follows_method(gpu):
    """WebPEncode calls of one picture size share a pooled engine: the ALPH
    effort must follow each call's method (alpha_enc.c:76,379), not the
    method of the call that created the engine"""
    img = alpha_frame(160, 96, 1)   # its ALPH stream differs for m0 / m2 / m6
    for m in (6, 2, 6, 0):
        data = gpu.encode_rgba(img, quality=75.0, method=m, exact=1)
        assert chunks(data)[b"ALPH"][1:] == M.encode(img[..., 3], method=m, alpha_plane=True), m


def test_model_alph_size_vs_reference():
    """ALPH sizes against the reference's (committed, lossless_kat.json):
    the logo plane takes a palette like the reference's"""
    k = json.load(open(os.path.join(ROOT, "tests", "golden", "lossless_kat.json")))
    for c in k["alph"]:
        img = (logo_frame if c["kind"] == "logo" else alpha_frame)(c["w"], c["h"], c["frame"])
        data, P = M.encode(img[..., 3], method=4, alpha_plane=True, return_parts=True)
        assert (P["palette"] is not None) == (c["kind"] == "logo")
        assert len(data) + 1 <= c["alph_size"] * c["tol"], (c, len(data) + 1)


def test_quantize_levels_model_matches_reference():
    """The oracle's QuantizeLevels restatement reproduces the level-reduced
    alpha planes the reference's own encodes decode to."""
    for case in kat()["cases"]:
        if case["alpha_quality"] >= 100:
            continue
        img = alpha_frame(case["w"], case["h"], case["frame"])
        q, _ = M.quantize_levels(img[..., 3], M.alpha_levels(case["alpha_quality"]))
        assert hashlib.sha256(q.tobytes()).hexdigest() == case["alpha_sha256"]
