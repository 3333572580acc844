import os, sys
sys.path.insert(0, os.getcwd())
import numpy as np, torch
import libwebp_amd as lw
from libwebp_amd.synth import syn_v1
for (w, h) in [(1, 1), (3, 5), (17, 9), (64, 48)]:
    enc = lw.GpuBatch(w, h, 1)
    enc.encode_host(syn_v1(w, h, 0)[None])
    print(w, h, len(enc.output(0)), flush=True)
    enc.close()
