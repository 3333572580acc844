"""trellis16 (lane-parallel) against the serial trellis_quant on random
blocks and cost tables (diagnostic build libwebp_amd_trace.so)."""
import ctypes as C
import json
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401  (one HIP runtime)
import libwebp_amd  # noqa: E402
lib = libwebp_amd.load()
out = (C.c_int * 1024)()
ok = lib.vp8g_trellis_selftest(int(sys.argv[1]) if len(sys.argv) > 1 else 4096, 12345, out)
o = list(out)
print(json.dumps({"ok": ok, "mismatch_blocks": o[0], "blocks": o[1], "first": {
    "group": o[2], "type": o[3], "ctx0": o[4], "lambda": o[5], "iter": o[6],
    "coeffs": o[8:24], "serial": o[24:40], "lane": o[40:56], "q": o[56:72],
    "sharpen": o[72:88], "nodes": [(v & 0xffff, (v >> 16) & 1, (v >> 17) & 1) for v in o[96:128]],
    "lanes": [dict(zip(["S0", "S1", "pv", "level0", "live1", "t00", "t01", "t10", "t11", "base0",
                        "base1", "nstar", "mstar", "nd", "cand", "RB"],
                       [int.from_bytes(C.c_int(o[128 + 32 * n + 2 * k]).value.to_bytes(4, "little", signed=True)
                                       + C.c_int(o[129 + 32 * n + 2 * k]).value.to_bytes(4, "little", signed=True),
                                       "little", signed=True) for k in range(16)]))
              for n in range(16)]}}))
