"""Regenerate tests/golden/alpha_kat.json with the reference build
(oracle/_ref/libwebp_ref.so, compiled from /root/reference by oracle/Makefile).
Dev container only:  python tests/golden/make_alpha_golden.py

Per case: the reference's 'VP8 ' chunk sha256 for the alpha frame of
tests/test_alpha.py:alpha_frame, and the sha256 of the RGB it decodes to.
"""
import ctypes
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from libwebp_amd import abi  # noqa: E402
from oracle import vp8l_model as M  # noqa: E402
from test_alpha import alpha_frame  # noqa: E402

CASES = [
    # api, w, h, frame, q, m, exact, alpha_compression, alpha_quality
    ("batch", 64, 48, 0, 75.0, 4, 0, 1, 100),
    ("batch", 333, 257, 5, 75.0, 4, 0, 1, 100),
    ("batch", 128, 96, 2, 90.0, 6, 1, 1, 100),
    ("batch", 200, 130, 3, 75.0, 4, 0, 0, 100),
    ("batch", 512, 384, 1, 75.0, 4, 0, 1, 100),
    ("webpencode", 160, 120, 4, 75.0, 4, 0, 1, 100),
    ("webpencode", 97, 61, 2, 80.0, 5, 0, 1, 100),
    ("webpencode", 96, 64, 6, 75.0, 3, 1, 0, 100),
    # alpha_quality < 100: QuantizeLevels (src/utils/quant_levels_utils.c)
    ("batch", 200, 130, 7, 75.0, 4, 0, 1, 50),
    ("batch", 333, 257, 8, 75.0, 4, 0, 1, 0),
    ("batch", 128, 96, 9, 75.0, 2, 0, 0, 85),
    ("webpencode", 160, 120, 10, 75.0, 4, 0, 1, 90),
    ("webpencode", 97, 61, 11, 60.0, 4, 1, 1, 20),
]


def main():
    lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "_ref", "libwebp_ref.so"))
    ref = abi.bind_encoder_api(lib)
    out = []
    for api, w, h, f, q, m, exact, ac, aq in CASES:
        img = alpha_frame(w, h, f)
        data, _ = abi.encode_rgba(ref, img, quality=q, method=m, exact=exact,
                                  alpha_compression=ac, alpha_quality=aq)
        ch = dict(M.riff_chunks(data))
        dec = M.ref_decode(lib, data)
        assert aq < 100 or (dec[..., 3] == img[..., 3]).all()
        out.append({"api": api, "w": w, "h": h, "frame": f, "q": q, "m": m, "exact": exact,
                    "alpha_compression": ac, "alpha_quality": aq,
                    "alpha_sha256": hashlib.sha256(dec[..., 3].tobytes()).hexdigest(),
                    "in_sha": hashlib.sha256(img.tobytes()).hexdigest()[:16],
                    "ref_size": len(data), "ref_alph_size": len(ch[b"ALPH"]),
                    "vp8_sha256": hashlib.sha256(ch[b"VP8 "]).hexdigest(),
                    "rgb_sha256": hashlib.sha256(dec[..., :3].tobytes()).hexdigest()})
    json.dump({"generator": "tests/golden/make_alpha_golden.py", "cases": out},
              open(os.path.join(HERE, "alpha_kat.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
