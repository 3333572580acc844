"""Minimal staged GPU check: one tiny frame, report the first failing call."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import libwebp_amd
from libwebp_amd.synth import syn_v1

lib = libwebp_amd.load()
print("devices", libwebp_amd.device_count(), flush=True)
w = h = int(sys.argv[1]) if len(sys.argv) > 1 else 16
img = syn_v1(w, h, 0)
enc = libwebp_amd.GpuBatch(w, h, 1)
print("batch created", flush=True)
try:
    enc.encode_host(img[None])
    print("encode ok, err=%d size=%d" % (enc.error(0), enc.output_size(0)), flush=True)
except Exception as e:
    print("FAILED:", e, flush=True)
print("last_error:", libwebp_amd.last_error(), flush=True)
