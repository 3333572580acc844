"""GPU debugging aid: tests/test_vp8l.py::test_gpu_near_lossless's first case
called directly (no pytest), printing the GPU and model sizes."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import libwebp_amd as gpu  # noqa: E402
import test_vp8l as T  # noqa: E402

img = T.lossless_picture("syn", 96, 80, 0)
for rep in range(3):
    enc = gpu.GpuBatch(96, 80, 1, quality=75.0, method=4, lossless=1, near_lossless=60)
    import torch
    buf = torch.from_numpy(np.ascontiguousarray(img[None])).to("cuda:0")
    torch.cuda.synchronize()
    enc.encode_device(buf.data_ptr(), 1)
    got = enc.output(0)
    enc.close()
    print("gpu", rep, len(got), flush=True)
print("model", len(T.M.encode(img, near_lossless_q=60)))
