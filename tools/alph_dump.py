"""Debug helper: encode the first batch case of tests/golden/alpha_kat.json on
the GPU and save the .webp (gpurun_out/alph_dump.webp)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402
import libwebp_amd as gpu  # noqa: E402
from libwebp_amd.synth import syn_v1  # noqa: E402
from test_alpha import alpha_frame  # noqa: E402

cases = [c for c in json.load(open(os.path.join(ROOT, "tests", "golden", "alpha_kat.json")))["cases"]
         if c["api"] == "batch"]
gpu.load()
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
for i, case in enumerate(cases):
    w, h, f = case["w"], case["h"], case["frame"]
    frames = np.stack([alpha_frame(w, h, f), syn_v1(w, h, f + 1)])
    enc = gpu.GpuBatch(w, h, 2, quality=case["q"], method=case["m"], exact=case["exact"],
                       alpha_compression=case["alpha_compression"],
                       alpha_quality=case["alpha_quality"])
    buf = torch.from_numpy(frames).to("cuda:0")
    torch.cuda.synchronize()
    enc.encode_device(buf.data_ptr(), 2)
    open(os.path.join(ROOT, "gpurun_out", "alph_dump%d.webp" % i), "wb").write(enc.output(0) or b"")
    enc.close()
    print(i, case["w"], case["h"], case["alpha_quality"])
