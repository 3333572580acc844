"""ctypes loader for the oracle (test infrastructure only; see vp8_oracle.h).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
this module.
"""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_lib = None


class Config(C.Structure):
    _fields_ = [("quality", C.c_float), ("method", C.c_int), ("segments", C.c_int),
                ("sns_strength", C.c_int), ("filter_strength", C.c_int),
                ("filter_sharpness", C.c_int), ("filter_type", C.c_int),
                ("partition_limit", C.c_int), ("preprocessing", C.c_int),
                ("emulate_jpeg_size", C.c_int), ("use_sharp_yuv", C.c_int),
                ("pass_", C.c_int), ("target_size", C.c_int), ("target_PSNR", C.c_float),
                ("qmin", C.c_int), ("qmax", C.c_int), ("autofilter", C.c_int),
                ("low_memory", C.c_int), ("partitions", C.c_int)]


class MBTrace(C.Structure):
    _fields_ = [("segment", C.c_uint8), ("type", C.c_uint8), ("uv_mode", C.c_uint8),
                ("skip", C.c_uint8), ("modes", C.c_uint8 * 16), ("alpha", C.c_uint8),
                ("pad", C.c_uint8 * 3), ("y_dc", C.c_int16 * 16),
                ("y_ac", C.c_int16 * 256), ("uv", C.c_int16 * 128)]


def lib():
    global _lib
    if _lib is None:
        path = os.path.join(_HERE, "_build", "libvp8oracle.so")
        if not os.path.exists(path):
            build()
        _lib = C.CDLL(path)
        _lib.vp8o_encode_rgba.restype = C.c_size_t
        _lib.vp8o_encode_yuv.restype = C.c_size_t
        _lib.vp8o_import_rgba.restype = C.c_int
        vp, i = C.c_void_p, C.c_int
        _lib.vp8o_import_rgba.argtypes = [vp, i, i, i, vp, vp, vp]
        _lib.vp8o_sharp_import_rgba.argtypes = [vp, i, i, i, vp, vp, vp]
        _lib.vp8o_import_rgba_dithered.argtypes = [vp, i, i, i, C.c_float, vp, vp, vp]
        _lib.vp8o_sharp_tables.argtypes = [vp, vp]
        _lib.vp8o_encode_yuv.argtypes = [vp, vp, vp, i, i, i, i, vp, vp, vp]
        _lib.vp8o_encode_rgba.argtypes = [vp, i, i, i, vp, vp]
        _lib.vp8o_analyze.argtypes = [vp, vp, vp, i, i, i, i, vp, vp, vp]
        _lib.vp8o_free.argtypes = [vp]
        _lib.vp8o_default_config.argtypes = [vp]
        _lib.odec_info.argtypes = [C.c_char_p, C.c_size_t] + [C.POINTER(C.c_int)] * 4
        _lib.odec_decode_rgba.argtypes = [C.c_char_p, C.c_size_t, vp]
        _lib.odec_decode_yuv.argtypes = [C.c_char_p, C.c_size_t, vp, vp, vp]
    return _lib


def build():
    import subprocess
    subprocess.check_call(
        ["make", "-s", "oracle",
         "CFLAGS=-O2 -fPIC -Wall -Wno-unused-function -Wno-missing-braces -I../libwebp_amd/csrc"],
        cwd=_HERE)


def config(quality=75.0, method=4, **kw):
    c = Config()
    lib().vp8o_default_config(C.byref(c))
    c.quality = quality
    c.method = method
    for k, v in kw.items():
        setattr(c, "pass_" if k == "pass" else k, v)
    return c


def import_rgba(rgba, sharp=False):
    """RGBA -> (Y, U, V). sharp=True: the iterative sharp-YUV conversion the
    reference applies for use_sharp_yuv (only from 4x4 up, like the
    reference; smaller pictures take the regular conversion)."""
    rgba = np.ascontiguousarray(rgba, np.uint8)
    h, w = rgba.shape[:2]
    uw, uh = (w + 1) // 2, (h + 1) // 2
    y = np.empty((h, w), np.uint8)
    u = np.empty((uh, uw), np.uint8)
    v = np.empty((uh, uw), np.uint8)
    if sharp and w >= 4 and h >= 4:
        if (rgba[..., 3] != 255).any():
            raise ValueError("non-opaque input is not restated by the oracle")
        fn = lib().vp8o_sharp_import_rgba
    else:
        fn = lib().vp8o_import_rgba
    ok = fn(rgba.ctypes.data, w, h, 4 * w, y.ctypes.data, u.ctypes.data, v.ctypes.data)
    if not ok:
        raise ValueError("non-opaque input is not restated by the oracle")
    return y, u, v


def encode_yuv(y, u, v, quality=75.0, method=4, trace=False, **kw):
    h, w = y.shape
    cfg = config(quality, method, **kw)
    out = C.POINTER(C.c_uint8)()
    nmb = ((w + 15) // 16) * ((h + 15) // 16)
    tr = (MBTrace * nmb)() if trace else None
    n = lib().vp8o_encode_yuv(y.ctypes.data, u.ctypes.data, v.ctypes.data, w, h,
                              y.strides[0], u.strides[0], C.byref(cfg), C.byref(out),
                              tr)
    if n == 0:
        raise RuntimeError("oracle encode failed")
    data = C.string_at(out, n)
    lib().vp8o_free(out)
    return (data, tr) if trace else data


def sharp_tables():
    g2l = np.empty(1026, np.uint32)
    l2g = np.empty(514, np.uint32)
    lib().vp8o_sharp_tables(g2l.ctypes.data, l2g.ctypes.data)
    return g2l, l2g


def import_rgba_dithered(rgba, dithering):
    """The dithered RGBA -> (Y, U, V) of WebPPictureARGBToYUVADithered."""
    rgba = np.ascontiguousarray(rgba, np.uint8)
    h, w = rgba.shape[:2]
    uw, uh = (w + 1) // 2, (h + 1) // 2
    y = np.empty((h, w), np.uint8)
    u = np.empty((uh, uw), np.uint8)
    v = np.empty((uh, uw), np.uint8)
    if not lib().vp8o_import_rgba_dithered(rgba.ctypes.data, w, h, 4 * w, dithering,
                                           y.ctypes.data, u.ctypes.data, v.ctypes.data):
        raise ValueError("non-opaque input is not restated by the oracle")
    return y, u, v


def encode_rgba(rgba, quality=75.0, method=4, **kw):
    sharp = bool(kw.pop("use_sharp_yuv", 0))
    if kw.get("preprocessing", 0) & 2 and not sharp:   # webp_enc.c:357-365
        x = np.float32(quality) / np.float32(100)
        x2 = x * x
        d = np.float32(1.0) + np.float32(0.5 - 1.0) * x2 * x2
        y, u, v = import_rgba_dithered(rgba, float(d))
    else:
        y, u, v = import_rgba(rgba, sharp=sharp)
    return encode_yuv(y, u, v, quality, method, **kw)


# ---- own WebP decoder (webp_dec.c): decode checks without reference code ----

def decode_info(data):
    """(width, height, has_alpha, lossless) of a .webp file."""
    w, h, a, ll = C.c_int(), C.c_int(), C.c_int(), C.c_int()
    if not lib().odec_info(data, len(data), C.byref(w), C.byref(h), C.byref(a), C.byref(ll)):
        raise ValueError("not a WebP bitstream the decoder understands")
    return w.value, h.value, bool(a.value), bool(ll.value)


def decode_rgba(data):
    """(H, W, 4) RGBA, what WebPDecodeRGBA returns (fancy upsampling for VP8)."""
    w, h, _, _ = decode_info(data)
    out = np.empty((h, w, 4), np.uint8)
    if not lib().odec_decode_rgba(data, len(data), out.ctypes.data):
        raise ValueError("decoder rejected the bitstream")
    return out


def decode_yuv(data):
    """(Y, U, V) planes of a lossy (VP8) .webp, cropped to the picture."""
    w, h, _, lossless = decode_info(data)
    if lossless:
        raise ValueError("decode_yuv needs a VP8 (lossy) bitstream")
    uw, uh = (w + 1) // 2, (h + 1) // 2
    y = np.empty((h, w), np.uint8)
    u = np.empty((uh, uw), np.uint8)
    v = np.empty((uh, uw), np.uint8)
    if not lib().odec_decode_yuv(data, len(data), y.ctypes.data, u.ctypes.data, v.ctypes.data):
        raise ValueError("decoder rejected the bitstream")
    return y, u, v
