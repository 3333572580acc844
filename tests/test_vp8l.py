"""Lossless (VP8L) path.

Parity contract (SURVEY.md §8(d), configs[4]): the bitstream must decode --
with the reference decoder -- to exactly the input pixels, and its size must
stay within VP8L_SIZE_TOL of the reference encoder's on the same frame. The
GPU bitstream is also checked bit for bit against oracle/vp8l_model.py, the
plain statement of the GPU algorithm (small frames), and the host header code
(vp8l_host.c) against the same model on CPU.
"""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

from libwebp_amd.synth import syn_v1
from oracle import vp8l_model as M

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# size of our lossless output relative to the reference encoder's (-lossless
# -m 4 -q 75) on syn-v1 frames (entropy-scored predictor and cross-colour
# search, oracle/vp8l_model.py): 0.994 at 512x512 (296,102 vs 297,970 B),
# 1.003 at 333x257 and 0.980 at 1080p f0 (2,292,116 vs 2,338,676 B)
VP8L_SIZE_TOL = 0.02
# per kind of picture (tests/golden/lossless_kat.json; every case's ratio in
# profiles/r6/lossless/ratios_r6q.json, tools/lossless_ratios.py): syn-v1,
# the 16-level spatial case and the tiled pictures within 2%; palettised
# graphics (glyph rows, rectangles; the hash-chain + cost-model parse, worst
# 0.998 since round 6's first-parse choice and 8-group cap), quantised syn-v1
# (worst 1.003) and the moderate-repeat pictures (worst 0.997) within 3%;
# text over a gradient within 5% (1080p 1.037: the reference spends 1,220
# code groups on it)
# (tiled syn-v1 / text over a gradient: more than 256 colours, long-range
# repeats: tests/golden/make_lossless_golden.py)
KIND_TOL = {"syn": 0.02, "g": 0.03, "q": 0.03, "q16": 0.02, "tile": 0.02, "text": 0.05,
            "mrep": 0.03}


def kind_tol(kind):
    if kind.startswith("mrep"):
        return KIND_TOL["mrep"]
    return KIND_TOL.get(kind, KIND_TOL.get(kind[0], KIND_TOL["syn"]))

CASES = [(64, 48, 0), (33, 17, 3), (1, 1, 0), (7, 5, 1), (2, 130, 4), (130, 3, 2)]


def ref_decoder():
    """the reference build (oracle/_ref), for comparisons with its ENCODER"""
    path = os.path.join(ROOT, "oracle", "_ref", "libwebp_ref.so")
    if not os.path.exists(path):
        pytest.skip("reference build oracle/_ref not present")
    return C.CDLL(path)


def decode(data):
    """decode through the own decoder (oracle/webp_dec.c, pinned against the
    reference decoder in tests/test_decoder.py)"""
    from oracle import oracle
    return oracle.decode_rgba(data)


def with_alpha(img, seed):
    rng = np.random.default_rng(seed)
    out = img.copy()
    out[..., 3] = rng.integers(0, 256, size=img.shape[:2], dtype=np.uint8)
    out[: img.shape[0] // 2, :, 3] = 255
    return out


# ------------------------------------------------------------------ model

@pytest.mark.parametrize("w,h,f", CASES)
def test_model_decodes_exact(w, h, f):
    img = syn_v1(w, h, f)
    assert np.array_equal(decode(M.encode(img)), img)


def same_but_transparent_rgb(dec, img):
    """decode equality where it is defined without `exact`: alpha everywhere,
    RGB where alpha != 0 (the predictor keeps only the alpha residual of a
    transparent pixel, predictor_enc.c:273-288)"""
    vis = img[..., 3] != 0
    return np.array_equal(dec[..., 3], img[..., 3]) and np.array_equal(dec[vis], img[vis])


def test_model_decodes_exact_alpha_and_methods():
    img = with_alpha(syn_v1(96, 80, 5), 3)
    assert (img[..., 3] == 0).any()
    for method in (0, 3, 4, 6):
        assert np.array_equal(decode(M.encode(img, method=method, exact=True)), img)
        assert same_but_transparent_rgb(decode(M.encode(img, method=method)), img)


def test_model_size_vs_reference_512():
    lib = ref_decoder()
    from libwebp_amd import abi
    ref = abi.bind_encoder_api(lib)
    img = syn_v1(512, 512, 0)
    ours = M.encode(img)
    theirs, _ = abi.encode_rgba(ref, img, quality=75.0, method=4, lossless=1, use_argb=True)
    assert len(ours) <= len(theirs) * (1 + VP8L_SIZE_TOL), (len(ours), len(theirs))


def lossless_cases(max_pixels):
    import json
    kat = json.load(open(os.path.join(ROOT, "tests", "golden", "lossless_kat.json")))
    return [c for c in kat["cases"] if c["w"] * c["h"] <= max_pixels]


def test_model_entropy_mode_and_size_vs_reference():
    """the model's entropy mode (transforms) equals the reference's on every
    fixture, its output decodes exactly and stays within the kind's size
    tolerance of the reference's (committed sizes, no reference needed)"""
    feats = {M.DIRECT: 0, M.SPATIAL: 3, M.SUBGREEN: 4, M.SPATIAL_SUBGREEN: 7, M.PALETTE: 8}
    for c in lossless_cases(600 * 600):
        img = lossless_picture(c["kind"], c["w"], c["h"], c["frame"])
        data, P = M.encode(img, return_parts=True)
        assert feats[P["mode"]] == c["features"], c
        if P["palette"] is not None:
            assert len(P["palette"]) == c["palette_size"], c
        assert np.array_equal(decode(data), img), c
        assert len(data) <= c["size"] * (1 + kind_tol(c["kind"])), (c, len(data))


def transparent_cases():
    import json
    kat = json.load(open(os.path.join(ROOT, "tests", "golden", "lossless_kat.json")))
    return kat["transparent"]


def zero_transparent(img):
    """WebPEncode's WebPReplaceTransparentPixels(pic, 0) without `exact`
    (src/enc/webp_enc.c:402-403)"""
    out = img.copy()
    out[out[..., 3] == 0] = 0
    return out


def test_model_transparent_matches_reference():
    """transparent areas without `exact`, incl. a border through pixel (0, 0)
    that AnalyzeEntropy's de-duplicated histograms never see: the alpha-0
    clean-up makes the decoded RGB depend on every tile's predictor, so the
    model takes the reference's own predictor search and its stream decodes
    to the reference encoder's pixels (committed SHA-256s of the reference's
    output decoded, tests/golden/make_lossless_golden.py)"""
    import hashlib
    for c in transparent_cases():
        img = zero_transparent(lossless_picture(c["kind"], c["w"], c["h"], c["frame"]))
        assert M.needs_exact_predictor(M.to_argb(img), 100, False), c
        data = M.encode(img)
        assert M.vp8l_transforms(data) == c["transforms"], c
        assert hashlib.sha256(decode(data).tobytes()).hexdigest() == c["decoded_sha256"], c
        assert len(data) <= c["size"] * 1.10, (c, len(data))


def test_model_near_lossless_matches_reference():
    """-near_lossless: the direct / subtract-green frames take the reference's
    VP8ApplyNearLossless (committed SHA-256s of its output), the spatial ones
    quantise inside the predictor; either way the stream opens with the
    reference's transforms and decodes to the reference encoder's pixels
    (committed SHA-256s of its decoded output; tests/golden/make_lossless_golden.py)"""
    import hashlib
    import json
    kat = json.load(open(os.path.join(ROOT, "tests", "golden", "lossless_kat.json")))
    for c in kat["near_lossless"]:
        img = lossless_picture(c["kind"], c["w"], c["h"], c["frame"])
        pre = M.near_lossless(M.to_argb(img), c["near_lossless"])
        assert hashlib.sha256(pre.astype("<u4").tobytes()).hexdigest() == c["argb_sha256"], c
        data = M.encode(img, near_lossless_q=c["near_lossless"])
        assert M.vp8l_transforms(data) == c["transforms"], c
        assert hashlib.sha256(decode(data).tobytes()).hexdigest() == c["decoded_sha256"], c


def test_model_residual_image_matches_reference():
    """residual_image == the reference's VP8LResidualImage: every tile's
    predictor and the residuals (near-lossless quantisation and alpha-0
    clean-up included) -- committed from the reference build"""
    import hashlib
    import json
    kat = json.load(open(os.path.join(ROOT, "tests", "golden", "lossless_kat.json")))
    for c in kat["residual_image"]:
        img = lossless_picture(c["kind"], c["w"], c["h"], c["frame"])
        argb = M.planes_argb(M.sub_green_planes(img, M.SUBGREEN if c["subtract_green"] else M.DIRECT))
        modes, res = M.residual_image(argb, c["tb"], False, c["near_lossless"], bool(c["exact"]),
                                      bool(c["subtract_green"]))
        assert modes.tolist() == c["modes"], c
        assert hashlib.sha256(res.astype("<u4").tobytes()).hexdigest() == c["residual_sha256"], c


def test_float_log_tables_match_reference():
    """kLog2Table / kSLog2Table (src/dsp/lossless_enc.c:28-224) are the float
    roundings the model and the engine's host tables compute"""
    import re
    src = "/root/reference/src/dsp/lossless_enc.c"
    if not os.path.exists(src):
        pytest.skip("reference sources absent")
    text = open(src).read()
    for name, mine in (("kLog2Table", M.LOG2_F32), ("kSLog2Table", M.SLOG2_F32)):
        body = re.search(r"const float " + name + r"\[LOG_LOOKUP_IDX_MAX\] = \{(.*?)\};", text, re.S)
        ref = np.array([np.float32(float(x)) for x in re.findall(r"([-0-9.]+)f", body.group(1))],
                       dtype=np.float32)
        assert len(ref) == 256 and np.array_equal(ref, mine), name


def test_host_float_tables_match_model(host_lib):
    host_lib.vp8l_float_tables.restype = C.POINTER(C.c_float)
    t = np.ctypeslib.as_array(host_lib.vp8l_float_tables(), shape=(512,))
    assert np.array_equal(t[:256], M.SLOG2_F32) and np.array_equal(t[256:], M.LOG2_F32)


def test_model_fast_slog2_matches_formula():
    """fast_slog2_f32 over the three ranges of FastSLog2Slow_C: table, the
    corrected approximation below 65536, libm log above"""
    v = np.array([0, 1, 2, 255, 256, 257, 1000, 4095, 4096, 65535, 65536, 70000, 2073600])
    got = M.fast_slog2_f32(v)
    assert got[0] == 0 and got[1] == 0 and got[2] == np.float32(2.0)
    for x, g in zip(v[4:], got[4:]):
        assert abs(float(g) - x * np.log2(x)) <= 0.02 * x, (x, g)


def test_prefix_and_distance_codes():
    for v in list(range(1, 70)) + [4095, 4096, 100000]:
        s, nb, e = M.prefix_encode(v)
        # GetCopyDistance (src/dec/vp8l_dec.c:159-168)
        if s < 4:
            back = s + 1
        else:
            xb = (s - 2) >> 1
            back = ((2 + (s & 1)) << xb) + e + 1
            assert xb == nb
        assert back == v
    for w in (1, 2, 7, 64, 1920):
        for d in M.candidate_distances(w):
            assert M.plane_code_to_distance(w, M.distance_code(w, d)) == d


# ------------------------------------------------------------------ host C vs model

class Params(C.Structure):
    _fields_ = [("w", C.c_int), ("h", C.c_int), ("n", C.c_int), ("tb", C.c_int),
                ("hb", C.c_int), ("k", C.c_int), ("dist", C.c_int * 4), ("dcode", C.c_int * 4),
                ("alpha", C.c_int), ("cache_bits", C.c_int), ("palette", C.c_int),
                ("xbits", C.c_int), ("ow", C.c_int), ("exact", C.c_int), ("nlq_bits", C.c_int),
                ("low_effort", C.c_int)]


class BW(C.Structure):
    _fields_ = [("buf", C.c_void_p), ("cap", C.c_size_t), ("pos", C.c_size_t),
                ("acc", C.c_uint64), ("used", C.c_int), ("nbits", C.c_uint64), ("oom", C.c_int)]


@pytest.fixture(scope="module")
def host_lib(tmp_path_factory):
    """vp8l_host.c compiled on its own (default visibility) for the test."""
    out = str(tmp_path_factory.mktemp("vp8l") / "libvp8lhost.so")
    src = os.path.join(ROOT, "libwebp_amd", "csrc", "host", "vp8l_host.c")
    subprocess.check_call(["gcc", "-O1", "-shared", "-fPIC", "-I",
                           os.path.join(ROOT, "libwebp_amd", "csrc"), src, "-o", out,
                           "-lm", "-lpthread"])
    lib = C.CDLL(out)
    vp = C.c_void_p
    lib.vp8l_build_header.restype = C.c_int
    lib.vp8l_build_header.argtypes = [vp, C.c_int, C.c_int, C.c_int, vp, C.c_int, vp, vp, vp, vp,
                                      vp, vp, vp]
    lib.vp8l_entropy_choice.argtypes = [vp, C.c_int, C.c_int]
    lib.vp8l_palette_order.argtypes = [vp, C.c_int]
    lib.vp8l_setup_palette_params.argtypes = [vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                              C.c_int]
    lib.vp8l_bw_finish.restype = C.c_size_t
    lib.vp8l_bw_finish.argtypes = [vp]
    lib.vp8l_bw_init.argtypes = [vp, C.c_size_t]
    lib.vp8l_bw_free.argtypes = [vp]
    lib.vp8l_setup_params.argtypes = [vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]
    lib.vp8l_setup_params_palette_hb.argtypes = [vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]
    return lib


def vp8l_ns():
    """the device layout: green alphabet sized for the largest cache"""
    return M.Alphabets(M.MAX_CACHE_BITS).ns


def to_device_layout(h, cache_bits):
    """model histogram rows (green alphabet 280 + 2^cache_bits) -> the device
    layout (green alphabet 280 + 2^MAX_CACHE_BITS)"""
    gs = M.Alphabets(cache_bits).gs
    pad = np.zeros(h.shape[:-1] + (M.Alphabets(M.MAX_CACHE_BITS).gs - gs,), h.dtype)
    return np.concatenate([h[..., :gs], pad, h[..., gs:]], axis=-1)


def alpha_plane(w, h, f):
    """A synthetic alpha plane: ramps, a transparent block and noise."""
    yy, xx = np.mgrid[0:h, 0:w]
    a = ((xx * 3 + yy + 17 * f) % 300).clip(0, 255).astype(np.uint8)
    a[: h // 3, : w // 3] = 0
    rng = np.random.default_rng(f)
    a[h // 2:, w // 2:] = rng.integers(0, 256, size=a[h // 2:, w // 2:].shape, dtype=np.uint8)
    return a


def graphics(w, h, ncol, seed):
    """A palettised test picture: ncol colours in rectangles and glyph rows."""
    rng = np.random.default_rng(seed)
    pal = rng.integers(0, 256, size=(ncol, 4), dtype=np.uint8)
    pal[:, 3] = 255
    idx = np.zeros((h, w), dtype=np.int64)
    for _ in range(60):
        x0, y0 = rng.integers(0, w), rng.integers(0, h)
        x1, y1 = x0 + rng.integers(4, w // 3 + 5), y0 + rng.integers(4, h // 3 + 5)
        idx[y0:y1, x0:x1] = rng.integers(0, ncol)
    for r in range(0, h, 24):
        glyph = rng.integers(0, 2, size=(8, w // 2)).repeat(2, axis=1)
        idx[r:r + 8, :glyph.shape[1]][glyph[:min(8, h - r)] == 1] = 0
    return pal[idx]


def quantized(w, h, levels, f):
    """syn-v1 with each channel cut to `levels` values (few hundred colours:
    the reference picks the direct mode on these)."""
    img = syn_v1(w, h, f).astype(np.int64)
    q = 256 // levels
    img[..., :3] = (img[..., :3] // q) * q
    return img.astype(np.uint8)


def tiled(w, h, f):
    """syn-v1 (thousands of colours) with long-range repeats: 64x64 tiles of
    the picture copied to other places, most of them rows away (the content
    only a hash-chain LZ77 search finds; backward_references_enc.c:259)."""
    img = syn_v1(w, h, f).copy()
    rng = np.random.default_rng(100 + f)
    T = 64
    srcs = [(int(rng.integers(0, max(1, h - T))), int(rng.integers(0, max(1, w - T))))
            for _ in range(4)]
    for ty in range(0, h - T + 1, T):
        for tx in range(0, w - T + 1, T):
            if (tx // T + 2 * (ty // T) + f) % 3 == 0:
                sy, sx = srcs[int(rng.integers(0, len(srcs)))]
                img[ty:ty + T, tx:tx + T] = img[sy:sy + T, sx:sx + T]
    return img


def moderate_repeats(w, h, f, every):
    """syn-v1 where about one 32x32 tile in `every` is a copy of a block at
    a random (unaligned) place: moderate long-range repeats that L0b's
    aligned window sampling does not see (the frame keeps the local parse)"""
    img = syn_v1(w, h, f).copy()
    rng = np.random.default_rng(300 + f)
    T = 32
    for ty in range(0, h - T + 1, T):
        for tx in range(0, w - T + 1, T):
            if rng.integers(0, every) == 0:
                sy, sx = int(rng.integers(0, h - T)), int(rng.integers(0, w - T))
                img[ty:ty + T, tx:tx + T] = img[sy:sy + T, sx:sx + T]
    return img


def text_on_gradient(w, h, f):
    """Anti-aliased 'text' over a colour gradient: a few hundred distinct
    8x12 glyphs set in lines (the same glyph repeats far apart), blended
    over a smooth background -- more than 256 colours, long-range repeats."""
    rng = np.random.default_rng(200 + f)
    yy, xx = np.mgrid[0:h, 0:w]
    bg = np.stack([(xx * 255) // max(1, w - 1), (yy * 255) // max(1, h - 1),
                   ((xx + yy) * 127) // max(1, w + h - 2) + 64], axis=-1).astype(np.int64)
    glyphs = rng.integers(0, 5, size=(40, 12, 8)) * 64   # coverage 0..256 in 5 steps
    glyphs = np.minimum(glyphs, 256)
    cov = np.zeros((h, w), dtype=np.int64)
    for r in range(4, h - 12, 16):
        x = 4
        while x + 8 < w:
            if rng.random() < 0.15:   # word gap
                x += 8
                continue
            cov[r:r + 12, x:x + 8] = glyphs[int(rng.integers(0, 40))]
            x += 9
    ink = np.array([20, 20, 40], dtype=np.int64)
    rgb = (bg * (256 - cov[..., None]) + ink * cov[..., None]) >> 8
    img = np.empty((h, w, 4), dtype=np.uint8)
    img[..., :3] = rgb
    img[..., 3] = 255
    return img


def transparent_border(w, h, f):
    """syn-v1 inside a fully transparent border that includes pixel (0, 0)
    (icons, sprites): every transparent pixel equals its left or upper
    neighbour, so AnalyzeEntropy's histograms never see one."""
    img = syn_v1(w, h, f).copy()
    b = 6 + f % 4
    img[:b, :, 3] = 0
    img[-b:, :, 3] = 0
    img[:, :b, 3] = 0
    img[:, -b:, 3] = 0
    return img


def transparent_sprite(w, h, f):
    """an opaque disc of syn-v1 on a transparent background (whose RGB is
    not zero: WebPEncode zeroes it unless `exact`)"""
    img = syn_v1(w, h, f).copy()
    yy, xx = np.mgrid[0:h, 0:w]
    r2 = (xx - w / 2) ** 2 + (yy - h / 2) ** 2
    img[..., 3] = np.where(r2 < (min(w, h) * 0.4) ** 2, 255, 0).astype(np.uint8)
    return img


def lossless_picture(kind, w, h, f):
    """syn-v1 ("syn"), palettised graphics ("g<colours>"), syn-v1 cut to
    <levels> values per channel ("q<levels>"), syn-v1 with repeated tiles
    ("tile"), text over a gradient ("text"), syn-v1 in a transparent border
    ("border"), a transparent-background sprite ("sprite") or syn-v1 with one
    unaligned copied tile in <every> ("mrep<every>")"""
    if kind == "syn":
        return syn_v1(w, h, f)
    if kind == "tile":
        return tiled(w, h, f)
    if kind.startswith("mrep"):
        return moderate_repeats(w, h, f, int(kind[4:]))
    if kind == "text":
        return text_on_gradient(w, h, f)
    if kind == "border":
        return transparent_border(w, h, f)
    if kind == "sprite":
        return transparent_sprite(w, h, f)
    if kind == "synt":   # syn-v1 with transparent (zeroed, as WebPEncode leaves them) and soft alpha
        img = syn_v1(w, h, f).copy()
        yy, xx = np.mgrid[0:h, 0:w]
        img[..., 3] = np.where(((xx // 8 + yy // 8) % 3) == 0, 128, 255)
        img[((xx * 7 + yy * 13 + f) % 11) < 2] = 0
        return img
    if kind[0] == "g":
        return graphics(w, h, int(kind[1:]), f)
    return quantized(w, h, int(kind[1:]), f)


def test_palette_helpers_match_model(host_lib):
    rng = np.random.default_rng(5)
    for n in (1, 2, 3, 17, 200, 256):
        cols = np.unique(rng.integers(0, 1 << 32, size=n, dtype=np.uint64).astype(np.uint32))
        if n == 3:   # monotone: stays sorted
            cols = np.array([0xff000000, 0xff010101, 0xff020202], dtype=np.uint32)
        want = M.minimize_deltas(cols)
        got = np.ascontiguousarray(rng.permutation(cols), dtype=np.uint32)
        host_lib.vp8l_palette_order(got.ctypes.data, len(got))
        assert got.tolist() == want
    for img in (syn_v1(64, 48, 0), graphics(96, 64, 40, 1), quantized(80, 60, 7, 2),
                graphics(90, 70, 200, 3), syn_v1(7, 5, 1)):
        h, w = img.shape[:2]
        argb = M.to_argb(img)
        ncol = len(np.unique(argb))
        npal = ncol if ncol <= M.MAX_PALETTE else 0
        tb = M.transform_bits(4, M.frame_histo_bits(4, w, h, npal))
        flat = argb.ravel()
        prev = np.concatenate([flat[:1], flat[:-1]])
        diff = M.sub_pixels_u32(flat, prev)
        keep = diff != 0
        keep[w:] &= flat[w:] != flat[:-w]
        hs = M.entropy_histograms(flat[keep].astype(np.int64), diff[keep].astype(np.int64))
        eh = np.ascontiguousarray(np.concatenate(hs), dtype=np.uint32)
        ntiles = M.sub_sample(w, tb) * M.sub_sample(h, tb)
        assert host_lib.vp8l_entropy_choice(eh.ctypes.data, npal, ntiles) == \
            M.analyze_entropy(argb, npal, tb)


@pytest.mark.parametrize("w,h,f,alpha,method,plane,kind", [
    (64, 48, 0, False, 4, False, "syn"), (33, 17, 3, False, 4, False, "syn"),
    (1, 1, 0, False, 4, False, "syn"), (256, 192, 2, False, 4, False, "syn"),
    (200, 130, 6, True, 4, False, "syn"), (160, 96, 1, False, 6, False, "syn"),
    (97, 61, 2, False, 3, False, "syn"), (120, 77, 1, False, 4, True, "syn"),
    (1, 1, 0, False, 4, True, "syn"), (96, 64, 1, False, 4, True, "logo"),
    (200, 130, 3, False, 4, True, "frame"), (96, 64, 1, False, 4, False, "g2"),
    (101, 67, 2, False, 4, False, "g4"), (90, 70, 3, False, 4, False, "g16"),
    (96, 64, 4, False, 4, False, "g200"), (80, 60, 0, False, 4, False, "q7"),
    (80, 60, 1, False, 4, False, "q4")])
def test_host_header_matches_model(host_lib, w, h, f, alpha, method, plane, kind):
    if plane and kind in ("logo", "frame"):   # the ALPH planes of tests/test_alpha.py
        from test_alpha import alpha_frame, logo_frame
        img = (logo_frame if kind == "logo" else alpha_frame)(w, h, f)[..., 3]
    elif plane:
        img = alpha_plane(w, h, f)
    elif kind == "syn":
        img = syn_v1(w, h, f)
    elif kind.startswith("g"):
        img = graphics(w, h, int(kind[1:]), f)
    else:
        img = quantized(w, h, int(kind[1:]), f)
    if alpha:
        img = with_alpha(img, f)
    _, P = M.encode(img, method=method, return_parts=True, alpha_plane=plane)
    p = Params()
    pal = P["palette"]
    if pal is not None:
        host_lib.vp8l_setup_palette_params(C.byref(p), w, h, 1, method, M.palette_xbits(len(pal)),
                                           int(plane))
        assert (p.hb, p.k, p.w) == (P["hb"], P["k"], P["argb"].shape[1])
    else:
        fits = plane or len(np.unique(M.to_argb(img))) <= M.MAX_PALETTE
        setup = host_lib.vp8l_setup_params_palette_hb if fits else host_lib.vp8l_setup_params
        setup(C.byref(p), w, h, 1, method, int(plane))
        assert (p.tb, p.hb, p.k) == (P["tb"], P["hb"], P["k"])
        assert p.low_effort == (method == 0)
    pw = P["argb"].shape[1]
    dists = M.candidate_distances(pw)
    assert list(p.dist)[:len(dists)] == dists
    assert list(p.dcode)[:len(dists)] == [M.distance_code(pw, d) for d in dists]
    ns = vp8l_ns()
    cb = P["cache_bits"]
    ntt = max(1, M.sub_sample(w, max(P["tb"], 2)) * M.sub_sample(h, max(P["tb"], 2)))
    modes = np.zeros(ntt, np.uint8)
    mult = np.zeros(ntt, np.uint32)
    if P["modes"] is not None:
        modes = np.ascontiguousarray(P["modes"], dtype=np.uint8)
        mult = np.ascontiguousarray((P["mult"][:, 0] & 255) | ((P["mult"][:, 1] & 255) << 8) |
                                    ((P["mult"][:, 2] & 255) << 16), dtype=np.uint32)
    hc = np.ascontiguousarray(to_device_layout(P["hc_raw"], cb), dtype=np.uint32)
    assert hc.shape == (16, ns)
    assign = np.ascontiguousarray(P["assign_raw"], dtype=np.uint8)
    ctab = np.zeros((16, ns), dtype=np.uint32)
    gtile = np.zeros(len(assign), dtype=np.uint8)
    palarr = np.ascontiguousarray(pal if pal is not None else [0], dtype=np.uint32)
    bw = BW()
    host_lib.vp8l_bw_init(C.byref(bw), C.c_size_t(1 << 16))
    ok = host_lib.vp8l_build_header(C.byref(p), int((img[..., 3] != 255).any()) if not plane else 0,
                                    P["mode"], cb, palarr.ctypes.data,
                                    len(pal) if pal is not None else 0, modes.ctypes.data,
                                    mult.ctypes.data, hc.ctypes.data, assign.ctypes.data,
                                    C.byref(bw), ctab.ctypes.data, gtile.ctypes.data)
    assert ok
    nbits = bw.nbits
    nb = host_lib.vp8l_bw_finish(C.byref(bw))
    got = C.string_at(bw.buf, nb)
    host_lib.vp8l_bw_free(C.byref(bw))
    assert nbits == P["header_bits"]
    assert got == P["header"]
    G = P["groups"]
    want = to_device_layout((P["code"] | (P["nb"] << 16)).astype(np.uint32), cb)
    assert np.array_equal(ctab[:G], want)
    assert np.array_equal(gtile, P["assign"].astype(np.uint8))


# ------------------------------------------------------------------ GPU

def gpu_encode(gpu, frames, method=4):
    import torch
    n, h, w, _ = frames.shape
    enc = gpu.GpuBatch(w, h, n, quality=75.0, method=method, lossless=1)
    buf = torch.from_numpy(np.ascontiguousarray(frames)).to("cuda:0")
    torch.cuda.synchronize()
    enc.encode_device(buf.data_ptr(), n)
    out = [enc.output(f) for f in range(n)]
    enc.close()
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("w,h,f", CASES + [(256, 192, 2)])
def test_gpu_matches_model(gpu, w, h, f):
    img = syn_v1(w, h, f)
    got = gpu_encode(gpu, img[None])[0]
    assert got == M.encode(img)


@pytest.mark.gpu
def test_gpu_alpha_methods_match_model(gpu):
    img = with_alpha(syn_v1(200, 130, 6), 6)
    for method in (3, 4, 6):
        assert gpu_encode(gpu, img[None], method=method)[0] == M.encode(img, method=method)


@pytest.mark.gpu
def test_gpu_low_methods_match_model(gpu):
    # methods 0-2: 64-pixel transform tiles (k_vp8l_transform with its
    # block-wide colour search; method 0: the reference's predictor choice, no
    # colour search), and 32-pixel ones at method 2 (k_vp8l_transform_w)
    for img in (with_alpha(syn_v1(200, 130, 6), 6), syn_v1(150, 100, 2)):
        for method in (0, 1, 2):
            assert gpu_encode(gpu, img[None], method=method)[0] == M.encode(img, method=method), \
                "method %d" % method


@pytest.mark.gpu
def test_gpu_batch_frames_match_model(gpu):
    frames = np.stack([syn_v1(160, 96, f) for f in range(5)])
    got = gpu_encode(gpu, frames)
    for f in range(5):
        assert got[f] == M.encode(frames[f]), "frame %d" % f


@pytest.mark.gpu
@pytest.mark.parametrize("kind,w,h,f", [("g2", 96, 64, 1), ("g4", 101, 67, 2), ("g16", 90, 70, 3),
                                        ("g200", 96, 64, 4), ("q7", 80, 60, 0), ("q4", 80, 60, 1),
                                        ("g16", 333, 31, 5), ("g2", 7, 130, 6)])
def test_gpu_entropy_modes_match_model(gpu, kind, w, h, f):
    """palette (each bundling), direct and subtract-green frames, and the
    per-frame colour-cache size, bit-exact with the model"""
    img = graphics(w, h, int(kind[1:]), f) if kind[0] == "g" else quantized(w, h, int(kind[1:]), f)
    got = gpu_encode(gpu, img[None])[0]
    assert got == M.encode(img)
    assert np.array_equal(decode(got), img)


@pytest.mark.gpu
def test_gpu_mixed_modes_batch(gpu):
    """one batch whose frames take different engines (spatial, direct,
    palettes of every bundling): routed back to their frame, bit-exact"""
    w, h = 96, 64
    frames = np.stack([syn_v1(w, h, 0), graphics(w, h, 2, 1), quantized(w, h, 7, 2),
                       graphics(w, h, 16, 3), graphics(w, h, 4, 4), syn_v1(w, h, 5),
                       graphics(w, h, 200, 6), graphics(w, h, 2, 7)])
    got = gpu_encode(gpu, frames)
    for f in range(len(frames)):
        assert got[f] == M.encode(frames[f]), "frame %d" % f


def test_repeat_test_separates_fixtures():
    """the repeat test (model: repeat_stats) sends the copied-tile pictures,
    and none of the other fixture kinds, to the hash-chain parse"""
    seen = set()
    for c in lossless_cases(1 << 30):
        k = (c["kind"], c["w"], c["h"], c["frame"])
        if k in seen or c["kind"][0] == "g":
            continue
        seen.add(k)
        img = lossless_picture(*k)
        assert M.repeat_heavy(img) == (c["kind"] == "tile"), (k, M.repeat_stats(img))


@pytest.mark.gpu
def test_gpu_repeat_routing_batch(gpu):
    """repeat-heavy frames (the lz sub-engine) beside spatial and palette
    frames in one batch: routed back to their frame, bit-exact with the model"""
    w, h = 320, 192
    frames = np.stack([tiled(w, h, 0), syn_v1(w, h, 1), graphics(w, h, 16, 2), tiled(w, h, 5),
                       tiled(w, h, 3)])   # (the last one has too few repeats: the local parse)
    assert [M.repeat_heavy(f) for f in frames] == [True, False, False, True, False]
    got = gpu_encode(gpu, frames)
    for f in range(len(frames)):
        assert got[f] == M.encode(frames[f]), "frame %d" % f


@pytest.mark.gpu
def test_gpu_1080p_decodes_exact_and_size(gpu):
    import json
    kat = json.load(open(os.path.join(ROOT, "tests", "golden", "kat.json")))
    sizes = {c["frame"]: c["size"] for c in kat.get("lossless", [])}
    frames = np.stack([syn_v1(1920, 1080, f) for f in range(3)])
    got = gpu_encode(gpu, frames)
    for f in range(3):
        assert np.array_equal(decode(got[f]), frames[f]), "frame %d" % f
        if f in sizes:
            assert len(got[f]) <= sizes[f] * (1 + VP8L_SIZE_TOL), (f, len(got[f]), sizes[f])


@pytest.mark.gpu
def test_gpu_1080p_palette_and_direct_sizes(gpu):
    """1080p palettised graphics and a quantised frame through one batch:
    decode-exact and within the kind's tolerance of the reference sizes"""
    cases = [c for c in lossless_cases(1 << 30) if c["kind"] != "syn"]
    big = [c for c in cases if c["w"] == 1920]
    for c in big:
        img = lossless_picture(c["kind"], c["w"], c["h"], c["frame"])
        got = gpu_encode(gpu, img[None])[0]
        assert np.array_equal(decode(got), img)
        if c["kind"] not in ("tile", "text"):   # test_gpu_1080p_repeat_sizes
            assert len(got) <= c["size"] * (1 + kind_tol(c["kind"])), (c, len(got))
    for c in cases:
        if c["w"] == 1920:
            continue
        img = lossless_picture(c["kind"], c["w"], c["h"], c["frame"])
        got = gpu_encode(gpu, img[None])[0]
        if c["w"] * c["h"] <= 200000:   # (the CPU model takes ~30 s on the larger ones)
            assert got == M.encode(img), c
        else:
            assert np.array_equal(decode(got), img), c
        assert len(got) <= c["size"] * (1 + kind_tol(c["kind"])), (c, len(got))


@pytest.mark.gpu
@pytest.mark.parametrize("kind", [
    "tile",    # repeat-heavy: the hash-chain parse (model 0.964x the reference; 1.29x before)
    "text"])   # direct-mode text over a gradient: 1.31x with the greedy parse, 1.037x with
               # the shortest-path parse over 32 plane codes + the colour cache (L3d)
def test_gpu_1080p_repeat_sizes(gpu, kind):
    """decode-exact always; size within the kind's tolerance of the reference"""
    c = [c for c in lossless_cases(1 << 30) if c["kind"] == kind and c["w"] == 1920][0]
    img = lossless_picture(c["kind"], c["w"], c["h"], c["frame"])
    got = gpu_encode(gpu, img[None])[0]
    assert np.array_equal(decode(got), img)
    assert len(got) <= c["size"] * (1 + kind_tol(c["kind"])), (c, len(got))


@pytest.mark.gpu
@pytest.mark.parametrize("kind,w,h,f,q", [("syn", 96, 80, 0, 60), ("syn", 200, 130, 2, 0),
                                          ("q7", 120, 90, 3, 40), ("syn", 64, 3, 1, 20),
                                          ("syn", 63, 63, 4, 0), ("g16", 96, 64, 3, 40)])
def test_gpu_near_lossless(gpu, kind, w, h, f, q):
    """near_lossless < 100 (VP8ApplyNearLossless preprocessing of direct /
    subtract-green frames, quantisation inside the predictor for spatial
    ones; palettes stay lossless): bit-exact with the model"""
    img = lossless_picture(kind, w, h, f)
    enc = gpu.GpuBatch(w, h, 1, quality=75.0, method=4, lossless=1, near_lossless=q)
    import torch
    buf = torch.from_numpy(np.ascontiguousarray(img[None])).to("cuda:0")
    torch.cuda.synchronize()
    enc.encode_device(buf.data_ptr(), 1)
    got = enc.output(0)
    enc.close()
    assert got == M.encode(img, near_lossless_q=q)
    data = gpu.encode_rgba(img, quality=75.0, method=4, lossless=1, use_argb=True, near_lossless=q)
    assert data == got   # opaque pictures: WebPEncode's transparent-pixel zeroing is a no-op
    # `exact` keeps the predictor's residuals plain, near-lossless included
    # (GetResidual's exact branch, predictor_enc.c:239-241)
    data = gpu.encode_rgba(img, quality=75.0, method=4, lossless=1, use_argb=True, exact=1,
                           near_lossless=q)
    assert data == M.encode(img, near_lossless_q=q, exact=True)


@pytest.mark.gpu
def test_gpu_near_lossless_decodes_like_reference(gpu):
    """WebPEncode -near_lossless on the GPU (spatial frames quantised inside
    the predictor, L1a / k_vp8l_resid_serial): the stream opens with the
    reference's transforms and decodes to the reference encoder's pixels
    (committed SHA-256s, tests/golden/make_lossless_golden.py)"""
    import hashlib
    import json
    kat = json.load(open(os.path.join(ROOT, "tests", "golden", "lossless_kat.json")))
    for c in kat["near_lossless"]:
        img = lossless_picture(c["kind"], c["w"], c["h"], c["frame"])
        data = gpu.encode_rgba(img, quality=75.0, method=4, lossless=1, use_argb=True,
                               near_lossless=c["near_lossless"])
        assert M.vp8l_transforms(data) == c["transforms"], c
        assert hashlib.sha256(decode(data).tobytes()).hexdigest() == c["decoded_sha256"], c
        assert data == M.encode(img, near_lossless_q=c["near_lossless"]), c


@pytest.mark.gpu
def test_gpu_transparent_no_exact(gpu):
    """WebPEncode -lossless without `exact` on pictures with transparent
    areas (a border through pixel (0, 0), a sprite on a transparent
    background): the engine's L0 counts transparent pixels over the whole
    picture and routes the frame to the reference's predictor search, so the
    stream equals the model's and decodes to the reference encoder's pixels"""
    import hashlib
    for c in transparent_cases():
        img = lossless_picture(c["kind"], c["w"], c["h"], c["frame"])
        data = gpu.encode_rgba(img, quality=75.0, method=4, lossless=1, use_argb=True)
        assert data == M.encode(zero_transparent(img)), c
        assert hashlib.sha256(decode(data).tobytes()).hexdigest() == c["decoded_sha256"], c


@pytest.mark.gpu
def test_gpu_webpencode_lossless_api(gpu):
    """WebPEncode with config.lossless (webp_enc.c:396-407): ARGB picture,
    transparent pixels zeroed unless `exact`; the one-shot
    WebPEncodeLosslessRGBA (picture_enc.c:285-297)."""
    img = with_alpha(syn_v1(160, 96, 4), 9)
    img[5, :40, 3] = 0   # fully transparent run
    data = gpu.encode_rgba(img, quality=75.0, method=4, lossless=1, use_argb=True, exact=1)
    assert data == M.encode(img, exact=True)
    assert np.array_equal(decode(data), img)
    # not exact: transparent pixels zeroed, then the predictor keeps only their
    # alpha residual (predictor_enc.c:273-288): RGB under alpha 0 is the prediction's
    data = gpu.encode_rgba(img, quality=75.0, method=4, lossless=1, use_argb=True)
    want = img.copy()
    want[want[..., 3] == 0] = 0
    assert data == M.encode(want)
    dec, opaque = decode(data), want[..., 3] != 0
    assert np.array_equal(dec[opaque], want[opaque]) and np.array_equal(dec[..., 3], want[..., 3])
    # one-shot API
    L = gpu.load()
    L.WebPEncodeLosslessRGBA.restype = C.c_size_t
    L.WebPEncodeLosslessRGBA.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int,
                                         C.POINTER(C.c_void_p)]
    out = C.c_void_p()
    a = np.ascontiguousarray(syn_v1(64, 48, 1))
    n = L.WebPEncodeLosslessRGBA(a.ctypes.data, 64, 48, 256, C.byref(out))
    assert n > 0
    got = C.string_at(out, n)
    L.WebPFree(out)
    assert np.array_equal(decode(got), a)
    assert got == M.encode(a, method=4)


def _dp_parse_py(argb, hit, bits, act, clen, ccode):
    """Pure-Python restatement of oracle/vp8l_dp.c (small pictures only)."""
    H, W = argb.shape
    dd = M.dp_candidates(W)
    dcodes = [M.distance_code(W, d) for d in dd]
    runs = M.match_lengths(argb, dd).reshape(len(dd), -1)
    px = argb.ravel().astype(np.int64)
    hv = hit.ravel() if bits else np.zeros(H * W, bool)
    for _ in range(2):
        (G, R, B, A, D), keys = M.dp_costs(argb, act, clen, ccode, bits)
        dcost = []
        for c in dcodes:
            s, nb, _ = M.prefix_encode(c)
            dcost.append(int(D[s]) + 256 * nb)
        lcost = [0] * 65
        for k in range(1, 65):
            s, nb, _ = M.prefix_encode(k)
            lcost[k] = int(G[256 + s]) + 256 * nb
        a2 = np.zeros(H * W, np.int64); c2 = np.zeros(H * W, np.int64); d2 = np.zeros(H * W, np.int64)
        for y in range(H):
            cost = [0] * (W + 1); chk = [1] * W; chc = [0] * W
            for j in range(W - 1, -1, -1):
                q = y * W + j
                a = int(px[q])
                if hv[q]:
                    best = cost[j + 1] + int(G[280 + keys[q]]) * 68 // 100
                else:
                    best = cost[j + 1] + (int(G[(a >> 8) & 255]) + int(R[(a >> 16) & 255]) +
                                          int(B[a & 255]) + int(A[a >> 24])) * 82 // 100
                bk, bc = 1, 0
                for k in range(2, 65):
                    if j + k > W:
                        break
                    cov = [(dcost[c], c) for c in range(len(dd)) if runs[c][q] >= k]
                    if not cov:
                        break
                    dc, cc = min(cov)
                    v = cost[j + k] + dc + lcost[k]
                    if v < best:
                        best, bk, bc = v, k, cc
                cost[j] = best; chk[j] = bk; chc[j] = bc
            j = 0
            while j < W:
                q = y * W + j
                if chk[j] >= 2:
                    a2[q] = 2; c2[q] = chk[j]; d2[q] = dcodes[chc[j]]
                    a2[q + 1:q + chk[j]] = 3
                    j += chk[j]
                else:
                    a2[q] = 1 if hv[q] else 0
                    j += 1
        act, clen, ccode = a2.reshape(H, W), c2.reshape(H, W), d2.reshape(H, W)
    return act, clen, ccode


@pytest.mark.parametrize("w,h,f,bits", [(24, 9, 0, 4), (17, 12, 1, 0), (5, 30, 2, 2), (1, 11, 3, 3)])
def test_dp_parse_c_matches_python(w, h, f, bits):
    """the shortest-path parse's C walk (oracle/vp8l_dp.c) equals its plain
    restatement, on pictures with repeats at small 2-D offsets"""
    rng = np.random.default_rng(f)
    base = rng.integers(0, 5, size=(h, w)).astype(np.uint32)
    img = np.zeros((h, w, 4), np.uint8)
    img[..., 1] = (base * 40).astype(np.uint8)
    img[..., 0] = ((base * 7) % 3 * 60).astype(np.uint8)
    img[..., 3] = 255
    img[h // 2:, : w // 2] = img[: h - h // 2, : w // 2]   # a repeat rows away
    argb = M.to_argb(img)
    flat = argb.ravel()
    minb = M.cache_minb(flat).reshape(h, w)
    hit = minb <= bits if bits else np.zeros((h, w), bool)
    dists = M.candidate_distances(w)
    act, clen, ccode = M.parse(argb, hit, dists)
    got = M.dp_parse(argb, hit, bits, act, clen, ccode)
    want = _dp_parse_py(argb, hit, bits, act, clen, ccode)
    for g, w_ in zip(got, want):
        assert np.array_equal(g, w_)


def test_dp_parse_text_size_vs_reference():
    """the direct-mode 1080p text fixture through the model with the
    shortest-path parse: within 5% of the reference's size (was 1.31x with
    the greedy parse)"""
    import json
    if not M.DP_ENABLED:
        pytest.skip("shortest-path parse switched off (DP_ENABLED)")
    c = [c for c in json.load(open(os.path.join(ROOT, "tests", "golden", "lossless_kat.json")))["cases"]
         if c["kind"] == "text" and c["w"] == 1920][0]
    img = lossless_picture(c["kind"], c["w"], c["h"], c["frame"])
    got = M.encode(img)
    assert len(got) <= c["size"] * 1.05, (len(got), c["size"])
