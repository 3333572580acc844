#!/usr/bin/env python3
"""Generate tests/golden/*.json from the reference libwebp built by
oracle/Makefile (oracle/_ref/libwebp_ref.so). Run in the dev container only:

    make -C oracle ref && python tests/golden/make_golden.py

Fixtures are data only: synthetic inputs are pinned by their SHA-256 (they are
regenerated from libwebp_amd.synth.syn_v1), expected outputs by size + SHA-256,
plus a few complete small bitstreams for debugging.
"""
import ctypes
import hashlib
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from libwebp_amd import abi  # noqa: E402
from libwebp_amd.synth import syn_v1  # noqa: E402

ref = abi.bind_encoder_api(ctypes.CDLL(os.path.join(ROOT, "oracle/_ref/libwebp_ref.so")))


def sha(b):
    return hashlib.sha256(b).hexdigest()


def case(w, h, f, **kw):
    img = syn_v1(w, h, f)
    out, st = abi.encode_rgba(ref, img, stats=True, **kw)
    return {"w": w, "h": h, "frame": f, "params": kw, "in_sha": sha(img.tobytes())[:16],
            "size": len(out), "sha256": sha(out),
            "block_count": list(st.block_count), "segment_quant": list(st.segment_quant),
            "segment_level": list(st.segment_level)}


def sharp_section():
    """use_sharp_yuv (sharpyuv/sharpyuv.c): plane hashes of
    WebPPictureSharpARGBToYUVA and full bitstreams of WebPEncode on an ARGB
    picture with use_sharp_yuv=1 (what cwebp -sharp_yuv does)."""
    import numpy as np
    sec = {"import": [], "encode": []}
    for (w, h, f) in [(4, 4, 0), (5, 7, 1), (3, 9, 2), (17, 9, 2), (64, 48, 3), (333, 257, 3),
                      (512, 512, 0), (1920, 1080, 0)]:
        y, u, v = abi.picture_yuv(ref, syn_v1(w, h, f), sharp=True)
        sec["import"].append({"w": w, "h": h, "frame": f, "y": sha(y.tobytes()),
                              "u": sha(u.tobytes()), "v": sha(v.tobytes())})
    # white noise: exercises the 10-bit clipping of the refinement
    img = np.random.RandomState(11).randint(0, 256, (130, 200, 4)).astype(np.uint8)
    img[..., 3] = 255
    y, u, v = abi.picture_yuv(ref, img, sharp=True)
    sec["noise_200x130_seed11"] = {"y": sha(y.tobytes()), "u": sha(u.tobytes()),
                                   "v": sha(v.tobytes())}
    for (w, h, f, q, m) in [(64, 48, 0, 75.0, 4), (333, 257, 5, 50.0, 6), (3, 3, 0, 75.0, 4),
                            (128, 77, 2, 90.0, 5), (512, 512, 0, 75.0, 4),
                            (1920, 1080, 0, 75.0, 4), (1920, 1080, 1, 75.0, 4)]:
        sec["encode"].append(case(w, h, f, quality=q, method=m, use_sharp_yuv=1))
    return sec


def tools_section():
    """Picture utilities (crop/rescale/YUVA->ARGB/distortion/cleanup/blend):
    the reference's answers on the fixed inputs of
    tests/test_picture_tools.tools_answers."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from test_picture_tools import tools_answers
    return tools_answers(ref)


def p0_section():
    """Partition-0 overflow retry (frame_enc.c:869-876): a 5120x5120 syn-v1
    frame at q95 m4 overflows the partition-0 estimate twice and is encoded in
    3 passes (pass count from the oracle restatement)."""
    from oracle import oracle
    c = case(5120, 5120, 0, quality=95.0, method=4)
    oracle.encode_rgba(syn_v1(5120, 5120, 0), quality=95.0, method=4)
    c["passes"] = oracle.lib().vp8o_last_pass_count()
    return [c]


SECTIONS = {"sharp": sharp_section, "tools": tools_section, "p0_overflow": p0_section}


def main():
    only = [a.split("=", 1)[1] for a in sys.argv if a.startswith("--only=")]
    if "--only-sharp" in sys.argv:
        only.append("sharp")
    if only:   # refresh some sections of an existing kat.json
        path = os.path.join(HERE, "kat.json")
        kat = json.load(open(path))
        for name in only:
            kat[name] = SECTIONS[name]()
        with open(path, "w") as fh:
            json.dump(kat, fh, indent=1)
        print("updated", only)
        return
    kat = {"survey": [], "sweep": [], "import": [], "bitstreams": {}}
    for f in (0, 7):
        kat["survey"].append(case(512, 512, f, quality=75.0, method=4))
    for f in range(8):
        kat["survey"].append(case(1920, 1080, f, quality=75.0, method=4))
    if "--big" in sys.argv:
        kat["survey"].append(case(4096, 4096, 0, quality=90.0, method=6))
    rnd = random.Random(1234)
    for _ in range(80):
        w = rnd.choice([1, 2, 3, 7, 16, 17, 33, 64, 100, 128, 200, 333])
        h = rnd.choice([1, 2, 5, 16, 31, 48, 77, 128, 257])
        kw = dict(quality=float(rnd.choice([0, 5, 30, 50, 75, 90, 98, 99, 100])),
                  method=rnd.choice([3, 4, 4, 5, 6]), segments=rnd.randint(1, 4),
                  sns_strength=rnd.choice([0, 25, 50, 80, 100]),
                  filter_strength=rnd.choice([0, 20, 60, 100]),
                  filter_sharpness=rnd.randint(0, 7), filter_type=rnd.randint(0, 1),
                  partition_limit=rnd.choice([0, 0, 50, 100]),
                  preprocessing=rnd.choice([0, 1]))
        kat["sweep"].append(case(w, h, rnd.randrange(64), **kw))
    for (w, h, f) in [(1, 1, 0), (3, 5, 1), (17, 9, 2), (333, 257, 3), (512, 512, 0),
                      (1920, 1080, 0), (1920, 1080, 1)]:
        y, u, v = abi.picture_yuv(ref, syn_v1(w, h, f))
        kat["import"].append({"w": w, "h": h, "frame": f, "y": sha(y.tobytes()),
                              "u": sha(u.tobytes()), "v": sha(v.tobytes())})
    for (w, h, f) in [(64, 48, 0), (333, 257, 5)]:
        out, _ = abi.encode_rgba(ref, syn_v1(w, h, f))
        name = "syn_%dx%d_f%d_q75_m4.webp" % (w, h, f)
        open(os.path.join(HERE, name), "wb").write(out)
        kat["bitstreams"][name] = sha(out)
    import subprocess
    import tempfile
    with tempfile.TemporaryDirectory() as td:
        exe = os.path.join(td, "probe")
        subprocess.check_call(["gcc", "-I/root/reference/src", os.path.join(ROOT, "tests", "abi_probe.c"),
                               "-o", exe])
        layout = json.loads(subprocess.check_output([exe]))
    with open(os.path.join(HERE, "abi_layout.json"), "w") as fh:
        json.dump(layout, fh, indent=1)
    kat["sharp"] = sharp_section()
    kat["tools"] = tools_section()
    kat["p0_overflow"] = p0_section()
    with open(os.path.join(HERE, "kat.json"), "w") as fh:
        json.dump(kat, fh, indent=1)
    print("wrote", len(kat["survey"]), "survey,", len(kat["sweep"]), "sweep cases")


if __name__ == "__main__":
    main()
