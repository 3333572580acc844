"""Intra-4 sub-stage split of the K3X main worker (diagnostic build
libwebp_amd/libwebp_amd_sub.so, -DK3_SUBPROF): one picture, row 0's main
worker's shader-clock cycles per stage summed over its MBs' searches.

usage: WEBP_AMD_LIB=libwebp_amd/libwebp_amd_sub.so python tools/k3x_sub.py W H [method] [quality]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import libwebp_amd  # noqa: E402

W, H = int(sys.argv[1]), int(sys.argv[2])
method = int(sys.argv[3]) if len(sys.argv) > 3 else 4
quality = float(sys.argv[4]) if len(sys.argv) > 4 else 75.0
names = ["edges+pred", "fdct", "quant/trellis", "idct+ballots", "distortion", "rate+stores",
         "bound+barrier+argmin", "commit"]
buf = torch.empty(W * H * 4, dtype=torch.uint8, device="cuda")
libwebp_amd.synth_device(buf.data_ptr(), W, H, 0, 1)
torch.cuda.synchronize()
enc = libwebp_amd.GpuBatch(W, H, 1, quality=quality, method=method)
enc.encode_device(buf.data_ptr(), 1)
enc.encode_device(buf.data_ptr(), 1)
t = enc.timings()
c = enc.stage_cycles(0)
mbw = (W + 15) // 16
tot = sum(c)
print("%dx%d q%g m%d: k_encode %.2f ms; row 0 main worker, cycles per MB (%d MBs):" %
      (W, H, quality, method, t[6] / 1e3, mbw))
for n, v in zip(names, c):
    print("  %-22s %7.0f  %5.1f%%" % (n, v / mbw, 100.0 * v / max(tot, 1)))
print("  total %.0f cycles per MB" % (tot / mbw))
