"""Lossless throughput of repeat-heavy frames (the hash-chain parse): n
copied-tile 1080p frames (tests/test_vp8l.py: tiled) through one engine,
against syn-v1 frames of the same size. Usage: python3 tools/lz_time.py [n]"""
import json, os, sys, time
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import libwebp_amd as gpu
from test_vp8l import tiled, syn_v1

n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
W, H = 1920, 1080
res = {}
for kind, fn in (("tile", tiled), ("syn", syn_v1)):
    base = [fn(W, H, f) for f in range(4)]
    frames = np.stack([base[i % 4] for i in range(n)])
    buf = torch.from_numpy(frames).to("cuda:0")
    enc = gpu.GpuBatch(W, H, n, quality=75.0, method=4, lossless=1)
    enc.encode_device(buf.data_ptr(), n)   # warm-up
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(3):
        enc.encode_device(buf.data_ptr(), n)
    dt = (time.perf_counter() - t) / 3
    sizes = [len(enc.output(f)) for f in range(4)]
    res[kind] = {"ms_per_call": round(dt * 1e3, 2), "mps": round(n * W * H / dt / 1e6, 1),
                 "sizes_first4": sizes}
    enc.close()
print(json.dumps(res))
