"""Per-MB side-info maps (picture.extra_info, cwebp -map, frame_enc.c:503-518)
of the reference encoder, types 1-5 and 7, as SHA-256s (dev container only:
needs oracle/_ref). usage: python tests/golden/make_extra_info_golden.py >
tests/golden/extra_info_kat.json"""
import ctypes as C
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from libwebp_amd import abi  # noqa: E402
from libwebp_amd.synth import syn_v1  # noqa: E402

CASES = [(96, 80, 0, dict(quality=75.0, method=4)),
         (333, 257, 1, dict(quality=60.0, method=6, segments=3)),
         (200, 120, 2, dict(quality=90.0, method=2)),
         (160, 96, 3, dict(quality=40.0, method=0, sns_strength=90, preprocessing=1)),
         (128, 128, 4, dict(quality=75.0, method=4, segments=1)),
         (257, 131, 5, dict(quality=30.0, method=3, pass_=1))]


def main():
    lib = abi.bind_encoder_api(C.CDLL(os.path.join(ROOT, "oracle", "_ref", "libwebp_ref.so")))
    out = []
    for w, h, f, kw in CASES:
        kw = {("pass" if k == "pass_" else k): v for k, v in kw.items()}
        img = syn_v1(w, h, f)
        maps = {}
        for t in (1, 2, 3, 4, 5, 7):
            data, m = abi.encode_rgba_map(lib, img, t, **kw)
            maps[str(t)] = hashlib.sha256(m).hexdigest()
        out.append({"w": w, "h": h, "frame": f, "params": kw,
                    "webp_sha256": hashlib.sha256(data).hexdigest(), "maps": maps})
    json.dump({"generator": "tests/golden/make_extra_info_golden.py (reference libwebp 1.3.2)",
               "cases": out}, sys.stdout, indent=1)


if __name__ == "__main__":
    main()
