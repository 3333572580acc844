"""The config-3 shard loop of tests/test_shards.py as a script that reports
each rank's step (time, frame errors, K3 error words) as it goes, so a stall
names its shard. Usage: python3 tools/shard_probe.py [ranks] [frames]"""
import os
import sys
import time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import libwebp_amd as gpu  # noqa: E402

W, H = 1920, 1080
ranks = int(sys.argv[1]) if len(sys.argv) > 1 else 8
B = int(sys.argv[2]) if len(sys.argv) > 2 else 256
fs = 4 * W * H
buf = torch.empty(B * fs, dtype=torch.uint8, device="cuda:0")
enc = gpu.GpuBatch(W, H, B, quality=75.0, method=4)
for r in range(ranks):
    gpu.synth_device(buf.data_ptr(), W, H, r * B, B)
    torch.cuda.synchronize()
    t = time.time()
    enc.encode_device(buf.data_ptr(), B)
    errs = sorted(set(enc.error(i) for i in range(B)))
    print("rank %d: %.3f s, errors %s" % (r, time.time() - t, errs), flush=True)
enc.close()
