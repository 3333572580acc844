"""Per-stage cycle split of the RD/token kernel (K3) on one batch."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import libwebp_amd

W, H = int(sys.argv[1]), int(sys.argv[2])
B = int(sys.argv[3]) if len(sys.argv) > 3 else 8
method = int(sys.argv[4]) if len(sys.argv) > 4 else 4
names = ["epoch+rowdone wait", "load+preds", "i16", "i4", "uv(+m5)", "info+sse+tokens",
         "ctx+boundary", "row-end fold"]
if os.environ.get("WEBP_AMD_LIB", "").endswith("_sub.so"):
    names = ["i4:decide+commit prev", "i4:edges+pred", "i4:fdct+quant+idct", "i4:distortion",
             "i4:rate+score", "i4:barrier", "-", "-"]
buf = torch.empty(B * W * H * 4, dtype=torch.uint8, device="cuda")
libwebp_amd.synth_device(buf.data_ptr(), W, H, 0, B)
torch.cuda.synchronize()
enc = libwebp_amd.GpuBatch(W, H, B, method=method)
enc.encode_device(buf.data_ptr(), B)
enc.encode_device(buf.data_ptr(), B)
t = enc.timings()
nmb = ((W + 15) // 16) * ((H + 15) // 16)
# the stamps are worker 0's: it encodes rows 0, NW, 2NW, ...
NW = {"2": 1, "3": 2, "4": 4, "5": 3}.get(os.environ.get("WEBP_AMD_K3", ""), 2 if method >= 5 else 4)
mbh = (H + 15) // 16
wmb = ((mbh + NW - 1) // NW) * ((W + 15) // 16)
c = enc.stage_cycles(0)
tot = sum(c)
if tot == 0:
    print("%dx%d batch %d m%d: k_encode %.1f ms (%.1f us/MB); stage cycles need a diagnostic build "
          "(WEBP_AMD_LIB=libwebp_amd/libwebp_amd_prof.so)" % (W, H, B, method, t[6] / 1e3, t[6] / nmb))
    sys.exit(0)
print("%dx%d batch %d m%d: k_encode %.1f ms (%.1f us/MB), tail %.1f ms" %
      (W, H, B, method, t[6] / 1e3, t[6] / nmb, t[4] / 1e3))
for n, v in zip(names, c):
    print("  %-20s %6.1f%%  %8.0f cycles per worker-MB" % (n, 100.0 * v / tot, v / wmb))
print("  total %.0f cycles per worker-MB (%d workers) -> %.1f us per worker-MB" %
      (tot / wmb, NW, t[6] / wmb))
