"""ctypes mirror of the libwebp encoder C ABI (version 0x020f).

The same structure definitions drive both our library (libwebp_amd.so) and the
reference build (oracle/_ref/libwebp_ref.so): the structs must be
byte-identical to src/webp/encode.h:95-153 (WebPConfig), :204-232
(WebPAuxStats), :242-247 (WebPMemoryWriter) and :300-364 (WebPPicture) of the
reference, which is what tests/test_abi.py checks against include/webp/encode.h.
"""
import ctypes as C

WEBP_ENCODER_ABI_VERSION = 0x020F

WEBP_PRESET_DEFAULT, WEBP_PRESET_PICTURE, WEBP_PRESET_PHOTO = 0, 1, 2
WEBP_PRESET_DRAWING, WEBP_PRESET_ICON, WEBP_PRESET_TEXT = 3, 4, 5

ENC_ERRORS = [
    "VP8_ENC_OK", "VP8_ENC_ERROR_OUT_OF_MEMORY",
    "VP8_ENC_ERROR_BITSTREAM_OUT_OF_MEMORY", "VP8_ENC_ERROR_NULL_PARAMETER",
    "VP8_ENC_ERROR_INVALID_CONFIGURATION", "VP8_ENC_ERROR_BAD_DIMENSION",
    "VP8_ENC_ERROR_PARTITION0_OVERFLOW", "VP8_ENC_ERROR_PARTITION_OVERFLOW",
    "VP8_ENC_ERROR_BAD_WRITE", "VP8_ENC_ERROR_FILE_TOO_BIG",
    "VP8_ENC_ERROR_USER_ABORT",
]


class WebPConfig(C.Structure):
    _fields_ = [(n, t) for n, t in [
        ("lossless", C.c_int), ("quality", C.c_float), ("method", C.c_int),
        ("image_hint", C.c_int), ("target_size", C.c_int),
        ("target_PSNR", C.c_float), ("segments", C.c_int),
        ("sns_strength", C.c_int), ("filter_strength", C.c_int),
        ("filter_sharpness", C.c_int), ("filter_type", C.c_int),
        ("autofilter", C.c_int), ("alpha_compression", C.c_int),
        ("alpha_filtering", C.c_int), ("alpha_quality", C.c_int),
        ("pass_", C.c_int), ("show_compressed", C.c_int),
        ("preprocessing", C.c_int), ("partitions", C.c_int),
        ("partition_limit", C.c_int), ("emulate_jpeg_size", C.c_int),
        ("thread_level", C.c_int), ("low_memory", C.c_int),
        ("near_lossless", C.c_int), ("exact", C.c_int),
        ("use_delta_palette", C.c_int), ("use_sharp_yuv", C.c_int),
        ("qmin", C.c_int), ("qmax", C.c_int)]]


class WebPAuxStats(C.Structure):
    _fields_ = [
        ("coded_size", C.c_int), ("PSNR", C.c_float * 5),
        ("block_count", C.c_int * 3), ("header_bytes", C.c_int * 2),
        ("residual_bytes", (C.c_int * 4) * 3), ("segment_size", C.c_int * 4),
        ("segment_quant", C.c_int * 4), ("segment_level", C.c_int * 4),
        ("alpha_data_size", C.c_int), ("layer_data_size", C.c_int),
        ("lossless_features", C.c_uint32), ("histogram_bits", C.c_int),
        ("transform_bits", C.c_int), ("cache_bits", C.c_int),
        ("palette_size", C.c_int), ("lossless_size", C.c_int),
        ("lossless_hdr_size", C.c_int), ("lossless_data_size", C.c_int),
        ("pad", C.c_uint32 * 2)]


class WebPMemoryWriter(C.Structure):
    _fields_ = [("mem", C.POINTER(C.c_uint8)), ("size", C.c_size_t),
                ("max_size", C.c_size_t), ("pad", C.c_uint32 * 1)]


class WebPPicture(C.Structure):
    pass


WebPWriterFunction = C.CFUNCTYPE(C.c_int, C.POINTER(C.c_uint8), C.c_size_t,
                                 C.POINTER(WebPPicture))
WebPProgressHook = C.CFUNCTYPE(C.c_int, C.c_int, C.POINTER(WebPPicture))

WebPPicture._fields_ = [
    ("use_argb", C.c_int), ("colorspace", C.c_int),
    ("width", C.c_int), ("height", C.c_int),
    ("y", C.POINTER(C.c_uint8)), ("u", C.POINTER(C.c_uint8)),
    ("v", C.POINTER(C.c_uint8)),
    ("y_stride", C.c_int), ("uv_stride", C.c_int),
    ("a", C.POINTER(C.c_uint8)), ("a_stride", C.c_int),
    ("pad1", C.c_uint32 * 2),
    ("argb", C.POINTER(C.c_uint32)), ("argb_stride", C.c_int),
    ("pad2", C.c_uint32 * 3),
    ("writer", C.c_void_p), ("custom_ptr", C.c_void_p),
    ("extra_info_type", C.c_int), ("extra_info", C.POINTER(C.c_uint8)),
    ("stats", C.POINTER(WebPAuxStats)), ("error_code", C.c_int),
    ("progress_hook", C.c_void_p), ("user_data", C.c_void_p),
    ("pad3", C.c_uint32 * 3), ("pad4", C.c_void_p), ("pad5", C.c_void_p),
    ("pad6", C.c_uint32 * 8), ("memory_", C.c_void_p),
    ("memory_argb_", C.c_void_p), ("pad7", C.c_void_p * 2)]


def bind_encoder_api(lib):
    """Declare argtypes/restype for the encode.h entry points on `lib`."""
    P = C.POINTER
    sigs = {
        "WebPGetEncoderVersion": (C.c_int, []),
        "WebPConfigInitInternal": (C.c_int, [P(WebPConfig), C.c_int, C.c_float, C.c_int]),
        "WebPConfigLosslessPreset": (C.c_int, [P(WebPConfig), C.c_int]),
        "WebPValidateConfig": (C.c_int, [P(WebPConfig)]),
        "WebPPictureInitInternal": (C.c_int, [P(WebPPicture), C.c_int]),
        "WebPPictureAlloc": (C.c_int, [P(WebPPicture)]),
        "WebPPictureFree": (None, [P(WebPPicture)]),
        "WebPPictureImportRGBA": (C.c_int, [P(WebPPicture), C.c_void_p, C.c_int]),
        "WebPPictureImportRGB": (C.c_int, [P(WebPPicture), C.c_void_p, C.c_int]),
        "WebPPictureImportBGRA": (C.c_int, [P(WebPPicture), C.c_void_p, C.c_int]),
        "WebPPictureSharpARGBToYUVA": (C.c_int, [P(WebPPicture)]),
        "WebPPictureSmartARGBToYUVA": (C.c_int, [P(WebPPicture)]),
        "WebPPictureARGBToYUVA": (C.c_int, [P(WebPPicture), C.c_int]),
        "WebPMemoryWriterInit": (None, [P(WebPMemoryWriter)]),
        "WebPMemoryWriterClear": (None, [P(WebPMemoryWriter)]),
        "WebPEncode": (C.c_int, [P(WebPConfig), P(WebPPicture)]),
        "WebPEncodeRGBA": (C.c_size_t, [C.c_void_p, C.c_int, C.c_int, C.c_int,
                                        C.c_float, P(P(C.c_uint8))]),
        "WebPFree": (None, [C.c_void_p]),
        "WebPPictureCopy": (C.c_int, [P(WebPPicture), P(WebPPicture)]),
        "WebPPlaneDistortion": (C.c_int, [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t,
                                          C.c_int, C.c_int, C.c_size_t, C.c_int,
                                          P(C.c_float), P(C.c_float)]),
        "WebPPictureDistortion": (C.c_int, [P(WebPPicture), P(WebPPicture), C.c_int,
                                            P(C.c_float)]),
        "WebPPictureCrop": (C.c_int, [P(WebPPicture), C.c_int, C.c_int, C.c_int, C.c_int]),
        "WebPPictureView": (C.c_int, [P(WebPPicture), C.c_int, C.c_int, C.c_int, C.c_int,
                                      P(WebPPicture)]),
        "WebPPictureIsView": (C.c_int, [P(WebPPicture)]),
        "WebPPictureRescale": (C.c_int, [P(WebPPicture), C.c_int, C.c_int]),
        "WebPPictureYUVAToARGB": (C.c_int, [P(WebPPicture)]),
        "WebPCleanupTransparentArea": (None, [P(WebPPicture)]),
        "WebPBlendAlpha": (None, [P(WebPPicture), C.c_uint32]),
        "WebPPictureHasTransparency": (C.c_int, [P(WebPPicture)]),
    }
    for name, (res, args) in sigs.items():
        if hasattr(lib, name):
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
    lib.WebPMemoryWrite_addr = C.cast(lib.WebPMemoryWrite, C.c_void_p).value
    return lib


def make_config(lib, quality=75.0, method=4, preset=WEBP_PRESET_DEFAULT, **kw):
    cfg = WebPConfig()
    if not lib.WebPConfigInitInternal(C.byref(cfg), preset, C.c_float(quality),
                                      WEBP_ENCODER_ABI_VERSION):
        raise RuntimeError("WebPConfigInitInternal failed")
    cfg.method = method
    for k, v in kw.items():
        setattr(cfg, "pass_" if k == "pass" else k, v)
    return cfg


def encode_rgba_map(lib, rgba, info_type, quality=75.0, method=4, **kw):
    """encode_rgba with picture.extra_info of type `info_type` (1..7, the
    per-MB map cwebp -map prints, src/enc/frame_enc.c:503-518): returns
    (bytes, map as bytes, mbw * mbh)."""
    h, w = rgba.shape[:2]
    n = ((w + 15) >> 4) * ((h + 15) >> 4)
    buf = (C.c_uint8 * n)(*([0xAA] * n))   # every entry must be written
    data, _ = encode_rgba(lib, rgba, quality, method, _extra_info=(info_type, buf), **kw)
    return data, bytes(buf)


def encode_rgba(lib, rgba, quality=75.0, method=4, stats=False, use_argb=None, _extra_info=None,
                progress=None, **kw):
    """Encode an (H, W, 4) uint8 array through `lib`'s WebPEncode().

    use_argb: import into the ARGB container first (what cwebp does for
    -sharp_yuv, examples/cwebp.c); defaults to on when use_sharp_yuv is set,
    since WebPEncode only re-converts an ARGB picture.

    progress: callable(percent) -> bool, installed as picture.progress_hook
    (a False return aborts the encode: VP8_ENC_ERROR_USER_ABORT).

    Returns (bytes, WebPAuxStats or None). Raises on encoder error.
    """
    import numpy as np
    rgba = np.ascontiguousarray(rgba, dtype=np.uint8)
    h, w = rgba.shape[:2]
    cfg = make_config(lib, quality, method, **kw)
    pic = WebPPicture()
    if not lib.WebPPictureInitInternal(C.byref(pic), WEBP_ENCODER_ABI_VERSION):
        raise RuntimeError("WebPPictureInitInternal failed")
    pic.width, pic.height = w, h
    if use_argb is None:
        use_argb = bool(kw.get("use_sharp_yuv", 0))
    pic.use_argb = int(use_argb)
    wrt = WebPMemoryWriter()
    lib.WebPMemoryWriterInit(C.byref(wrt))
    pic.writer = lib.WebPMemoryWrite_addr
    pic.custom_ptr = C.cast(C.pointer(wrt), C.c_void_p)
    st = WebPAuxStats() if stats else None
    if st is not None:
        pic.stats = C.pointer(st)
    hook = None
    if progress is not None:
        hook = WebPProgressHook(lambda pct, _pic: 1 if progress(pct) else 0)
        pic.progress_hook = C.cast(hook, C.c_void_p)
    if _extra_info is not None:
        pic.extra_info_type = _extra_info[0]
        pic.extra_info = C.cast(_extra_info[1], C.POINTER(C.c_uint8))
    try:
        if not lib.WebPPictureImportRGBA(C.byref(pic), rgba.ctypes.data, 4 * w):
            raise RuntimeError("import failed: %s" % ENC_ERRORS[pic.error_code])
        if not lib.WebPEncode(C.byref(cfg), C.byref(pic)):
            why = ""
            if hasattr(lib, "WebPGpuLastError"):   # libwebp_amd's engine diagnostics
                why = " (%s)" % lib.WebPGpuLastError().decode(errors="replace")
            raise RuntimeError("WebPEncode failed: %s%s" % (ENC_ERRORS[pic.error_code], why))
        data = C.string_at(wrt.mem, wrt.size)
    finally:
        lib.WebPPictureFree(C.byref(pic))
        lib.WebPMemoryWriterClear(C.byref(wrt))
    return data, st


def picture_yuv(lib, rgba, sharp=False):
    """Run WebPPictureImportRGBA through `lib` and return (Y, U, V) arrays.
    sharp=True: import into ARGB, then WebPPictureSharpARGBToYUVA."""
    import numpy as np
    rgba = np.ascontiguousarray(rgba, dtype=np.uint8)
    h, w = rgba.shape[:2]
    pic = WebPPicture()
    lib.WebPPictureInitInternal(C.byref(pic), WEBP_ENCODER_ABI_VERSION)
    pic.width, pic.height = w, h
    pic.use_argb = 1 if sharp else 0
    try:
        if not lib.WebPPictureImportRGBA(C.byref(pic), rgba.ctypes.data, 4 * w):
            raise RuntimeError("import failed")
        if sharp and not lib.WebPPictureSharpARGBToYUVA(C.byref(pic)):
            raise RuntimeError("sharp conversion failed")
        uw, uh = (w + 1) // 2, (h + 1) // 2
        y = np.ctypeslib.as_array(pic.y, shape=(h * pic.y_stride,)).reshape(h, pic.y_stride)[:, :w].copy()
        u = np.ctypeslib.as_array(pic.u, shape=(uh * pic.uv_stride,)).reshape(uh, pic.uv_stride)[:, :uw].copy()
        v = np.ctypeslib.as_array(pic.v, shape=(uh * pic.uv_stride,)).reshape(uh, pic.uv_stride)[:, :uw].copy()
    finally:
        lib.WebPPictureFree(C.byref(pic))
    return y, u, v
