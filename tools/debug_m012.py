"""GPU debug: methods 0-2 outputs (GPU vs oracle) over tests/test_methods012.py
CASES; prints the VP8 header fields of mismatching pairs."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tools"), os.path.join(ROOT, "tests")]
import libwebp_amd as gpu  # noqa: E402
from libwebp_amd.synth import syn_v1  # noqa: E402
from oracle import oracle  # noqa: E402
from vp8_header import parse  # noqa: E402
from test_methods012 import CASES  # noqa: E402

for w, h, f, kw in CASES:
    if w * h > 300000:
        continue
    img = syn_v1(w, h, f)
    g, st = gpu.encode_rgba(img, stats=True, **kw)
    o = oracle.encode_rgba(img, **kw)
    po = parse(o)
    print(kw, w, h, len(g), len(o), "OK" if g == o else "DIFF", list(st.block_count),
          "skip" if po.get("skip") else "noskip")
