"""Debug helper: encode one synthetic lossless picture on the GPU and save
the bitstream (gpurun_out/vp8l_dump.webp) for comparison with the model."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch  # noqa: E402
import libwebp_amd as gpu  # noqa: E402
from test_vp8l import graphics, quantized, gpu_encode  # noqa: E402

kind, w, h, f = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
img = graphics(w, h, int(kind[1:]), f) if kind[0] == "g" else quantized(w, h, int(kind[1:]), f)
gpu.load()
out = gpu_encode(gpu, img[None])[0]
os.makedirs("gpurun_out", exist_ok=True)
open("gpurun_out/vp8l_dump.webp", "wb").write(out)
print("wrote", len(out))
