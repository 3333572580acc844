"""The own WebP decoder (oracle/webp_dec.c): decode
checks on the GPU box need no reference code. Pinned here against the
reference decoder built from /root/reference (oracle/_ref) on streams the
REFERENCE encoder wrote over its option space, and against the reference's
own decode fixture (examples/test.webp -> test_ref.ppm, copied as data to
tests/golden/ref_examples/)."""
import ctypes as C
import os
import random

import numpy as np
import pytest

from libwebp_amd import abi
from libwebp_amd.synth import syn_v1
from oracle import oracle
from oracle import vp8l_model as M

HERE = os.path.dirname(os.path.abspath(__file__))


def ref_yuv(lib, data):
    """WebPDecodeYUV of the reference build: (Y, U, V) cropped planes."""
    lib.WebPDecodeYUV.restype = C.c_void_p
    lib.WebPDecodeYUV.argtypes = [C.c_char_p, C.c_size_t, C.POINTER(C.c_int), C.POINTER(C.c_int),
                                  C.POINTER(C.c_void_p), C.POINTER(C.c_void_p),
                                  C.POINTER(C.c_int), C.POINTER(C.c_int)]
    lib.WebPFree.argtypes = [C.c_void_p]
    w, h, ys, uvs = C.c_int(), C.c_int(), C.c_int(), C.c_int()
    u, v = C.c_void_p(), C.c_void_p()
    y = lib.WebPDecodeYUV(data, len(data), C.byref(w), C.byref(h), C.byref(u), C.byref(v),
                          C.byref(ys), C.byref(uvs))
    assert y
    W, H = w.value, h.value
    uw, uh = (W + 1) // 2, (H + 1) // 2
    Y = np.frombuffer(C.string_at(y, ys.value * H), np.uint8).reshape(H, ys.value)[:, :W].copy()
    U = np.frombuffer(C.string_at(u.value, uvs.value * uh), np.uint8).reshape(uh, uvs.value)[:, :uw].copy()
    V = np.frombuffer(C.string_at(v.value, uvs.value * uh), np.uint8).reshape(uh, uvs.value)[:, :uw].copy()
    lib.WebPFree(y)
    return Y, U, V


def with_alpha(img, seed):
    rng = np.random.default_rng(seed)
    out = img.copy()
    a = rng.integers(0, 256, size=img.shape[:2], dtype=np.uint8)
    a[: img.shape[0] // 3] = 255
    a[:, : img.shape[1] // 4] = (np.arange(img.shape[0])[:, None] * 7 % 256).astype(np.uint8)
    out[..., 3] = a
    return out


def test_reference_example_fixture():
    """examples/test.webp decodes to examples/test_ref.ppm (the reference's
    own decode known answer; 'within +-1 LSB' in SURVEY 8(c), exact here)"""
    data = open(os.path.join(HERE, "golden", "ref_examples", "test.webp"), "rb").read()
    ppm = open(os.path.join(HERE, "golden", "ref_examples", "test_ref.ppm"), "rb").read()
    parts = ppm.split(b"\n", 3)
    assert parts[0] == b"P6"
    w, h = [int(t) for t in parts[1].split()]
    want = np.frombuffer(parts[3][: w * h * 3], np.uint8).reshape(h, w, 3)
    got = oracle.decode_rgba(data)
    assert got.shape[:2] == (h, w)
    # test_ref.ppm predates the current YUV->RGB rounding: the reference's own
    # decoder differs from it by up to 1 LSB too (and equals ours exactly,
    # test_reference_example_vs_reference_decoder)
    assert np.abs(got[..., :3].astype(int) - want).max() <= 1


def test_reference_example_vs_reference_decoder(ref_lib):
    data = open(os.path.join(HERE, "golden", "ref_examples", "test.webp"), "rb").read()
    assert np.array_equal(oracle.decode_rgba(data), M.ref_decode(ref_lib, data))


def test_lossy_random_reference_streams(ref_lib):
    """reference-encoded VP8 streams over methods 0-6, segments, filters
    (simple / normal, sharpness, strength), token partitions, skip flags,
    sizes 1..150: RGBA and YUV equal to the reference decoder's"""
    rnd = random.Random(11)
    for i in range(40):
        w, h = rnd.randint(1, 150), rnd.randint(1, 150)
        kw = dict(quality=float(rnd.randint(0, 100)), method=rnd.randint(0, 6),
                  segments=rnd.randint(1, 4), sns_strength=rnd.randint(0, 100),
                  filter_strength=rnd.randint(0, 100), filter_sharpness=rnd.randint(0, 7),
                  filter_type=rnd.randint(0, 1), partitions=rnd.randint(0, 3),
                  autofilter=rnd.randint(0, 1) if i % 5 == 0 else 0)
        img = syn_v1(w, h, rnd.randrange(100))
        data, _ = abi.encode_rgba(ref_lib, img, **kw)
        assert np.array_equal(oracle.decode_rgba(data), M.ref_decode(ref_lib, data)), (w, h, kw)
        for a, b in zip(oracle.decode_yuv(data), ref_yuv(ref_lib, data)):
            assert np.array_equal(a, b), (w, h, kw)


def test_alpha_reference_streams(ref_lib):
    """VP8X + ALPH + VP8: raw and VP8L-compressed alpha, every alpha filter,
    level reduction; RGBA equal to the reference decoder's"""
    rnd = random.Random(5)
    for i in range(16):
        w, h = rnd.randint(1, 120), rnd.randint(1, 120)
        kw = dict(quality=float(rnd.randint(10, 100)), method=rnd.randint(0, 6),
                  alpha_compression=rnd.randint(0, 1), alpha_filtering=rnd.randint(0, 2),
                  alpha_quality=rnd.choice([100, 100, 60, 20]), exact=1)
        img = with_alpha(syn_v1(w, h, i), i)
        data, _ = abi.encode_rgba(ref_lib, img, **kw)
        got = oracle.decode_rgba(data)
        assert np.array_equal(got, M.ref_decode(ref_lib, data)), (w, h, kw)
        if kw["alpha_quality"] == 100:
            assert np.array_equal(got[..., 3], img[..., 3])


@pytest.mark.parametrize("kind", ["syn", "palette", "alpha"])
def test_lossless_reference_streams(ref_lib, kind):
    """VP8L streams of the reference encoder (predictor / cross-colour /
    subtract-green / colour-indexing transforms, colour cache, meta Huffman
    codes, LZ77 plane codes) decode to the exact input pixels"""
    rnd = random.Random({"syn": 1, "palette": 2, "alpha": 3}[kind])
    for i in range(8):
        w, h = rnd.randint(1, 140), rnd.randint(1, 140)
        img = syn_v1(w, h, i)
        if kind == "palette":   # <= 16 colours: colour indexing with bit packing
            ncol = rnd.choice([2, 3, 4, 11, 16, 40])
            pal = np.random.default_rng(i).integers(0, 256, size=(ncol, 4), dtype=np.uint8)
            pal[:, 3] = 255
            img = pal[(img[..., 0].astype(int) * 7 + img[..., 1]) % ncol]
        elif kind == "alpha":
            img = with_alpha(img, i)
        kw = dict(quality=float(rnd.randint(0, 100)), method=rnd.randint(0, 6), lossless=1,
                  exact=1)
        data, _ = abi.encode_rgba(ref_lib, img, use_argb=True, **kw)
        got = oracle.decode_rgba(data)
        assert np.array_equal(got, img), (kind, w, h, kw)
        assert np.array_equal(got, M.ref_decode(ref_lib, data)), (kind, w, h, kw)


def test_own_encoder_streams():
    """streams of the repo's own CPU models: VP8L model streams decode to the
    exact input; oracle VP8 streams decode to planes of the picture's size"""
    for w, h, f in [(64, 48, 0), (33, 17, 3), (1, 1, 0), (130, 3, 2)]:
        img = syn_v1(w, h, f)
        assert np.array_equal(oracle.decode_rgba(M.encode(img)), img)
        y, u, v = oracle.decode_yuv(oracle.encode_rgba(img))
        assert y.shape == (h, w) and u.shape == ((h + 1) // 2, (w + 1) // 2)


def test_rejects_garbage():
    with pytest.raises(ValueError):
        oracle.decode_rgba(b"RIFF\x04\x00\x00\x00WEBPjunk")
    data = oracle.encode_rgba(syn_v1(16, 16, 0))
    with pytest.raises(ValueError):
        oracle.decode_rgba(data[:20])


def test_decode_kat_own_decoder():
    """the own decoder reproduces the committed reference-decoded hashes
    (tests/golden/decode_kat.json) from the oracle's bitstreams, which equal
    the reference encoder's (tests/test_oracle.py)"""
    import hashlib
    import json
    for c in json.load(open(os.path.join(HERE, "golden", "decode_kat.json")))["cases"]:
        if c["w"] * c["h"] > 600000:
            continue   # 1080p cases: GPU test only (the oracle encode takes seconds)
        data = oracle.encode_rgba(syn_v1(c["w"], c["h"], c["frame"]), quality=c["q"],
                                  method=c["m"])
        assert hashlib.sha256(data).hexdigest() == c["webp_sha256"]
        y, u, v = oracle.decode_yuv(data)
        assert hashlib.sha256(y.tobytes() + u.tobytes() + v.tobytes()).hexdigest() == c["yuv_sha256"]
        assert hashlib.sha256(oracle.decode_rgba(data).tobytes()).hexdigest() == c["rgba_sha256"]
