"""Decoded-pixel known answers (run in the dev container, where the reference
build oracle/_ref exists): the reference encoder's SURVEY 8(d) bitstreams
decoded by the reference decoder (WebPDecodeYUV planes, WebPDecodeRGBA
pixels), as SHA-256s. tests/test_gpu_parity.py decodes the GPU's bitstreams
with the own decoder (oracle/webp_dec.c) and compares against these.

usage: python tests/golden/make_decode_golden.py > tests/golden/decode_kat.json"""
import ctypes as C
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from libwebp_amd import abi  # noqa: E402
from libwebp_amd.synth import syn_v1  # noqa: E402
from oracle import vp8l_model as M  # noqa: E402
from test_decoder import ref_yuv  # noqa: E402


def main():
    lib = C.CDLL(os.path.join(ROOT, "oracle", "_ref", "libwebp_ref.so"))
    enc = abi.bind_encoder_api(lib)
    out = []
    for w, h, f in [(512, 512, 0), (1920, 1080, 0), (1920, 1080, 1), (333, 257, 2)]:
        data, _ = abi.encode_rgba(enc, syn_v1(w, h, f), quality=75.0, method=4)
        y, u, v = ref_yuv(lib, data)
        rgba = M.ref_decode(lib, data)
        out.append({"w": w, "h": h, "frame": f, "q": 75.0, "m": 4,
                    "webp_sha256": hashlib.sha256(data).hexdigest(),
                    "yuv_sha256": hashlib.sha256(y.tobytes() + u.tobytes() + v.tobytes()).hexdigest(),
                    "rgba_sha256": hashlib.sha256(rgba.tobytes()).hexdigest()})
    json.dump({"generator": "tests/golden/make_decode_golden.py (reference libwebp 1.3.2 "
                            "encode + decode, oracle/_ref)", "cases": out}, sys.stdout, indent=1)


if __name__ == "__main__":
    main()
