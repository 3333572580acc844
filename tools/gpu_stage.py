"""Minimal staged GPU check: one tiny frame through the device-input path,
then through the host-input path. Exits non-zero at the first failure so a
GPU command chained with && stops there."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch          # first: our library then binds to torch's HIP runtime
torch.cuda.init()
import libwebp_amd
from libwebp_amd.synth import syn_v1
from oracle import oracle

lib = libwebp_amd.load()
print("devices", libwebp_amd.device_count(), flush=True)
w = h = int(sys.argv[1]) if len(sys.argv) > 1 else 16
img = syn_v1(w, h, 0)
ref = oracle.encode_rgba(img)

dev = torch.device("cuda", 0)
buf = torch.empty(w * h * 4, dtype=torch.uint8, device=dev)
libwebp_amd.synth_device(buf.data_ptr(), w, h, 0, 1)
torch.cuda.synchronize()
print("synth ok, matches numpy:", bool((buf.cpu().numpy() == img.reshape(-1)).all()), flush=True)

enc = libwebp_amd.GpuBatch(w, h, 1)
print("batch created", flush=True)
try:
    enc.encode_device(buf.data_ptr(), 1)
    out = enc.output(0)
    print("device path ok: size=%d oracle=%d equal=%s" % (len(out), len(ref), out == ref),
          flush=True)
except Exception as e:
    print("FAILED device path:", e, flush=True)
    sys.exit(1)
try:
    enc.encode_host(img[None])
    out = enc.output(0)
    print("host path ok: size=%d equal=%s" % (len(out), out == ref), flush=True)
except Exception as e:
    print("FAILED host path:", e, flush=True)
    sys.exit(1)
print("last_error:", libwebp_amd.last_error(), flush=True)
