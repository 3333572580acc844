"""GPU debugging aid: encode one lossless test picture through GpuBatch
with LIBWEBP_AMD_VP8L_DUMP set (slot 0's residual image after L1, parse
ops, cache bits, predictor modes, multipliers and the serial flag go to
gpurun_out/<tag>/dump.*) and save the stream.
Usage: python3 tools/vp8l_dump_case.py <tag> <kind> <w> <h> <frame> [near_lossless] [method]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

tag, kind, w, h, f = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
q = int(sys.argv[6]) if len(sys.argv) > 6 else 100
method = int(sys.argv[7]) if len(sys.argv) > 7 else 4
out = os.path.join(ROOT, "gpurun_out", tag)
os.makedirs(out, exist_ok=True)
if not tag.endswith("_nodump"):
    os.environ["LIBWEBP_AMD_VP8L_DUMP"] = os.path.join(out, "dump")
import torch  # noqa: E402
import libwebp_amd as gpu  # noqa: E402
from test_vp8l import lossless_picture  # noqa: E402
img = lossless_picture(kind, w, h, f)
enc = gpu.GpuBatch(w, h, 1, quality=75.0, method=method, lossless=1, near_lossless=q)
buf = torch.from_numpy(np.ascontiguousarray(img[None])).to("cuda:0")
torch.cuda.synchronize()
enc.encode_device(buf.data_ptr(), 1)
open(os.path.join(out, "stream.webp"), "wb").write(enc.output(0))
enc.close()
print("ok", len(open(os.path.join(out, "stream.webp"), "rb").read()))
