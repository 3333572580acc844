"""Regenerate tests/golden/multipass_kat.json with the reference build
(oracle/_ref/libwebp_ref.so, compiled from /root/reference by oracle/Makefile).
Dev container only:  python tests/golden/make_multipass_golden.py

Multi-pass lossy encodes (VP8EncTokenLoop with config->pass > 1,
src/enc/frame_enc.c:783-894): plain extra passes, the target_size and
target_PSNR searches (InitPassStats / ComputeNextQ, :47-80) and qmin/qmax.
Per case: syn-v1 input hash, the reference's output size and sha256.
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
from test_multipass import CASES  # noqa: E402
from libwebp_amd.synth import syn_v1  # noqa: E402


def main():
    ref = abi.bind_encoder_api(ctypes.CDLL(os.path.join(ROOT, "oracle", "_ref",
                                                        "libwebp_ref.so")))
    out = []
    for w, h, f, kw in CASES:
        img = syn_v1(w, h, f)
        data, st = abi.encode_rgba(ref, img, stats=True, **kw)
        out.append({"w": w, "h": h, "frame": f, "params": kw,
                    "in_sha": hashlib.sha256(img.tobytes()).hexdigest()[:16],
                    "size": len(data), "sha256": hashlib.sha256(data).hexdigest(),
                    "psnr_y": round(float(st.PSNR[0]), 3)})
    json.dump({"generator": "tests/golden/make_multipass_golden.py", "cases": out},
              open(os.path.join(HERE, "multipass_kat.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
