#!/usr/bin/env python3
"""Known answers for the frames bench.py checks inside its timed batch
(BASELINE.json configs[1] and configs[2]: 1920x1080 syn-v1, -q 75 -m 4, rank r
encodes frames [256r, 256r + 256)). Generated with the reference libwebp built
by oracle/Makefile (oracle/_ref/libwebp_ref.so). Dev container only:

    make -C oracle ref && python tests/golden/make_shard_golden.py

Writes tests/golden/shard_kat.json: {frame: {"size", "sha256", "in_sha"}} for
the first, a middle and the last frame of each of the 8 ranks' shards, plus
frames 0..7 (the SURVEY.md 8(d) table).
"""
import ctypes
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from libwebp_amd import abi  # noqa: E402
from libwebp_amd.synth import syn_v1  # noqa: E402

W, H, Q, M, PER_RANK, RANKS = 1920, 1080, 75.0, 4, 256, 8


def frames():
    fs = set(range(8))
    for r in range(RANKS):
        fs |= {PER_RANK * r, PER_RANK * r + 131, PER_RANK * r + PER_RANK - 1}
    return sorted(fs)


def main():
    ref = abi.bind_encoder_api(ctypes.CDLL(os.path.join(ROOT, "oracle", "_ref",
                                                        "libwebp_ref.so")))
    out = {}
    for f in frames():
        img = syn_v1(W, H, f)
        data, _ = abi.encode_rgba(ref, img, quality=Q, method=M)
        out[str(f)] = {"size": len(data), "sha256": hashlib.sha256(data).hexdigest(),
                       "in_sha": hashlib.sha256(img.tobytes()).hexdigest()[:16]}
    json.dump({"generator": "tests/golden/make_shard_golden.py", "width": W, "height": H,
               "quality": Q, "method": M, "frames": out},
              open(os.path.join(HERE, "shard_kat.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
