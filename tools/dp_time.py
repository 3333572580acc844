"""Lossless encode of a batch of 1080p text-over-gradient frames (direct
mode: the shortest-path parse runs on every frame), timed; sizes against
the reference's for the committed fixture frame.
usage: python tools/dp_time.py [frames]"""
import json
import os
import sys
import time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np  # noqa: E402
import libwebp_amd as gpu  # noqa: E402
from test_vp8l import text_on_gradient  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
W, H = 1920, 1080
frames = np.stack([text_on_gradient(W, H, 2 + (i % 4)) for i in range(n)])
enc = gpu.GpuBatch(W, H, n, quality=75.0, method=4, lossless=1)
enc.encode_host(frames)
t = time.time()
enc.encode_host(frames)
dt = time.time() - t
sizes = [len(enc.output(i)) for i in range(n)]
print(json.dumps({"frames": n, "seconds": round(dt, 4), "mp_per_s": round(n * W * H / dt / 1e6, 1),
                  "size_f2": sizes[0], "reference_f2": 1555708,
                  "ratio_f2": round(sizes[0] / 1555708, 4)}))
