"""Time one small batch through the GPU engine (HBM-resident syn-v1 frames):
K3X (frames split over CUs) vs the one-workgroup K3, selected by
WEBP_AMD_K3X=0/1 in the environment.

usage: python tools/k3x_time.py W H N QUALITY METHOD [REPS]
prints one JSON line: ms per call (median), k_encode ms from the engine's
HIP events, and the SHA-256 of frame 0."""
import hashlib
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import libwebp_amd
    w, h, n, q, m = (int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), float(sys.argv[4]),
                     int(sys.argv[5]))
    reps = int(sys.argv[6]) if len(sys.argv) > 6 else 3
    buf = torch.empty(n * w * h * 4, dtype=torch.uint8, device="cuda:0")
    libwebp_amd.synth_device(buf.data_ptr(), w, h, 0, n)
    torch.cuda.synchronize()
    enc = libwebp_amd.GpuBatch(w, h, n, quality=q, method=m)
    times, k3 = [], []
    for _ in range(reps):
        t0 = time.perf_counter()
        enc.encode_device(buf.data_ptr(), n)
        times.append((time.perf_counter() - t0) * 1e3)
        k3.append(enc.timings())
    out = enc.output(0)
    times.sort()
    print(json.dumps({"w": w, "h": h, "n": n, "q": q, "m": m,
                      "k3x": os.environ.get("WEBP_AMD_K3X", "1"),
                      "ms_median": round(times[len(times) // 2], 2),
                      "ms_all": [round(t, 2) for t in times],
                      "timings_last": [round(t, 3) for t in k3[-1]],
                      "mp_s": round(w * h * n / (times[len(times) // 2] * 1e3), 2),
                      "size0": len(out), "sha0": hashlib.sha256(out).hexdigest()}), flush=True)
    enc.close()


if __name__ == "__main__":
    main()
