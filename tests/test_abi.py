"""The C-ABI boundary: libwebp_amd.so loads on a CPU-only host, exports every
entry point declared in include/webp/*.h, and its public structs are
byte-identical to the reference's (tests/golden/abi_layout.json, measured on
the reference header src/webp/encode.h)."""
import ctypes
import json
import os
import re
import subprocess
import tempfile

import pytest

import libwebp_amd
from libwebp_amd import abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    names = set()
    for hdr in ("types.h", "encode.h", "encode_gpu.h"):
        text = open(os.path.join(ROOT, "include", "webp", hdr)).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        text = re.sub(r"^\s*#.*$", "", text, flags=re.M)   # drop macro definitions
        for m in re.finditer(r"WEBP_EXTERN\s+[^;{(]*?\b(\w+)\s*\(", text):
            names.add(m.group(1))
    return names


def test_library_exports_every_declared_symbol():
    lib = libwebp_amd.load()
    names = declared_symbols()
    assert "WebPEncode" in names and "WebPGpuBatchEncodeRGBA" in names
    missing = [n for n in sorted(names) if not hasattr(lib, n)]
    assert not missing, missing


def test_struct_layout_matches_reference():
    want = json.load(open(os.path.join(ROOT, "tests", "golden", "abi_layout.json")))
    with tempfile.TemporaryDirectory() as td:
        exe = os.path.join(td, "probe")
        subprocess.check_call(["gcc", "-I" + os.path.join(ROOT, "include"),
                               os.path.join(ROOT, "tests", "abi_probe.c"), "-o", exe])
        got = json.loads(subprocess.check_output([exe]))
    assert got == want


def test_ctypes_mirror_matches_header():
    want = json.load(open(os.path.join(ROOT, "tests", "golden", "abi_layout.json")))
    assert ctypes.sizeof(abi.WebPConfig) == want["sizeof.WebPConfig"]
    assert ctypes.sizeof(abi.WebPPicture) == want["sizeof.WebPPicture"]
    assert ctypes.sizeof(abi.WebPAuxStats) == want["sizeof.WebPAuxStats"]
    assert abi.WebPPicture.memory_.offset == want["WebPPicture.memory_"]
    assert abi.WebPPicture.writer.offset == want["WebPPicture.writer"]


def test_config_api_matches_reference_semantics(ref_lib):
    lib = libwebp_amd.load()
    for preset in range(6):
        for q in (0.0, 37.5, 75.0, 100.0):
            a, b = abi.WebPConfig(), abi.WebPConfig()
            assert lib.WebPConfigInitInternal(ctypes.byref(a), preset, q, abi.WEBP_ENCODER_ABI_VERSION)
            assert ref_lib.WebPConfigInitInternal(ctypes.byref(b), preset, q,
                                                  abi.WEBP_ENCODER_ABI_VERSION)
            assert bytes(a) == bytes(b), (preset, q)
    c = abi.WebPConfig()
    # ABI major mismatch is rejected
    assert not lib.WebPConfigInitInternal(ctypes.byref(c), 0, 75.0, 0x0300)
    # validation agrees on out-of-range fields
    for field, val in [("quality", 101.0), ("method", 7), ("segments", 0), ("pass_", 11),
                       ("filter_sharpness", 8), ("partitions", 4), ("qmin", 50)]:
        a = abi.make_config(lib)
        setattr(a, field, val)
        if field == "qmin":
            a.qmax = 40
        b = abi.WebPConfig.from_buffer_copy(bytes(a))
        assert lib.WebPValidateConfig(ctypes.byref(a)) == ref_lib.WebPValidateConfig(ctypes.byref(b)) == 0


def test_encoder_version():
    assert libwebp_amd.load().WebPGetEncoderVersion() == 0x010302


def test_memory_writer_and_picture_alloc():
    lib = libwebp_amd.load()
    pic = abi.WebPPicture()
    assert lib.WebPPictureInitInternal(ctypes.byref(pic), abi.WEBP_ENCODER_ABI_VERSION)
    pic.width, pic.height = 33, 17
    assert lib.WebPPictureAlloc(ctypes.byref(pic))
    assert pic.y_stride == 33 and pic.uv_stride == 17
    lib.WebPPictureFree(ctypes.byref(pic))
    assert not pic.y
    pic.width = 0
    assert not lib.WebPPictureAlloc(ctypes.byref(pic))
    assert pic.error_code == 5   # VP8_ENC_ERROR_BAD_DIMENSION


def test_encode_without_gpu_fails_loudly():
    if libwebp_amd.device_count() > 0:
        pytest.skip("GPU present")
    from libwebp_amd.synth import syn_v1
    with pytest.raises(RuntimeError):
        libwebp_amd.encode_rgba(syn_v1(32, 32, 0))
    with pytest.raises(RuntimeError):
        libwebp_amd.GpuBatch(32, 32, 1)
