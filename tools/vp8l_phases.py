"""Phase cycle split of the lossless transform kernels (L1a k_vp8l_predsel,
L1 k_vp8l_transform) on one batch; needs the diagnostic build
(WEBP_AMD_LIB=libwebp_amd/libwebp_amd_prof.so, -DVP8L_PS_PROF).
Usage: python3 tools/vp8l_phases.py W H B [method]"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import libwebp_amd  # noqa: E402

W, H, B = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
method = int(sys.argv[4]) if len(sys.argv) > 4 else 4
buf = torch.empty(B * W * H * 4, dtype=torch.uint8, device="cuda")
libwebp_amd.synth_device(buf.data_ptr(), W, H, 0, B)
torch.cuda.synchronize()
enc = libwebp_amd.GpuBatch(W, H, B, method=method, lossless=1)
lib = libwebp_amd.load()
fn = lib.vp8l_prof_phase_cycles
fn.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
out = (C.c_ulonglong * 16)()
enc.encode_device(buf.data_ptr(), B)
fn(out, 1)
enc.encode_device(buf.data_ptr(), B)
fn(out, 1)
tb = 5 if method in (2, 3, 4) else (4 if method > 4 else 6)
ntt = ((W + (1 << tb) - 1) >> tb) * ((H + (1 << tb) - 1) >> tb)
names = {0: "L1a load", 1: "L1a maxd/flags", 2: "L1a histograms", 3: "L1a terms",
         4: "L1a chains", 5: "L1a select+acc", 6: "L1 load", 7: "L1 predictor choice",
         8: "L1 residuals", 9: "L1 colour search (rest)", 10: "L1 final residuals",
         11: "  cc zero", 12: "  cc pixels", 13: "  cc bins"}
for i, n in names.items():
    print("%-18s %12.0f clk per tile" % (n, out[i] / (B * ntt)))
