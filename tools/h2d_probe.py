"""H2D upload rate from pinned host memory (the bench's host-input leg):
one copy of B x 1080p RGBA frames on 1, 2, 4, 8 streams at once (the copy
split into equal chunks), alone and beside a long-running kernel."""
import json
import sys
import time

import torch

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
nbytes = B * 1920 * 1080 * 4
dev = torch.device("cuda", 0)
src = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
src.fill_(7)
dst = torch.empty(nbytes, dtype=torch.uint8, device=dev)
out = {}
for ns in (1, 2, 4, 8):
    streams = [torch.cuda.Stream(dev) for _ in range(ns)]
    chunk = (nbytes + ns - 1) // ns
    for rep in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i, s in enumerate(streams):
            lo, hi = i * chunk, min(nbytes, (i + 1) * chunk)
            with torch.cuda.stream(s):
                dst[lo:hi].copy_(src[lo:hi], non_blocking=True)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
    out["h2d_streams_%d_GBs" % ns] = round(nbytes / el / 1e9, 2)
# device -> host
for ns in (1, 4):
    streams = [torch.cuda.Stream(dev) for _ in range(ns)]
    chunk = (nbytes + ns - 1) // ns
    for rep in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i, s in enumerate(streams):
            lo, hi = i * chunk, min(nbytes, (i + 1) * chunk)
            with torch.cuda.stream(s):
                src[lo:hi].copy_(dst[lo:hi], non_blocking=True)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
    out["d2h_streams_%d_GBs" % ns] = round(nbytes / el / 1e9, 2)
out["bytes"] = nbytes
print(json.dumps(out))
