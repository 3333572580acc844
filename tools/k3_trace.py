"""Per-worker wait / stage accounting of K3 (diagnostic build
libwebp_amd/libwebp_amd_trace.so, -DK3_TRACE): one batch of syn-v1 frames,
then the counters of every workgroup's workers summed and split.

usage: WEBP_AMD_LIB=libwebp_amd/libwebp_amd_trace.so \
       python tools/k3_trace.py W H B [method] [quality] [json_out]"""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import libwebp_amd  # noqa: E402

SLOTS = ["refresher_wait", "epoch_wait", "row_wait", "fold_wait", "fold", "replay", "n_replay",
         "refresh", "mb", "i4", "i16", "n_mb", "total", "n_row_waits", "tokens", "uv"]
W, H, B = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
method = int(sys.argv[4]) if len(sys.argv) > 4 else 4
quality = float(sys.argv[5]) if len(sys.argv) > 5 else 75.0
out_json = sys.argv[6] if len(sys.argv) > 6 else None
buf = torch.empty(B * W * H * 4, dtype=torch.uint8, device="cuda")
libwebp_amd.synth_device(buf.data_ptr(), W, H, 0, B)
torch.cuda.synchronize()
enc = libwebp_amd.GpuBatch(W, H, B, quality=quality, method=method)
enc.encode_device(buf.data_ptr(), B)
enc.encode_device(buf.data_ptr(), B)
t = enc.timings()
lib = libwebp_amd.load()
if hasattr(lib, "vp8g_k3_check"):   # check build: the index-check record of both calls
    ck = (C.c_ulonglong * 8)()
    lib.vp8g_k3_check.restype = C.c_int
    assert lib.vp8g_k3_check(ck)
    rec = {"failed_checks": int(ck[0])}
    if ck[0]:
        rec.update(site=int(ck[1]), workgroup=int(ck[2]), thread=int(ck[3]), mb=int(ck[4]),
                   value=int(ck[5]), bound=int(ck[6]))
    print("K3_CHECK", json.dumps(rec), flush=True)
    hang = (C.c_uint32 * (1024 * 4 * 10))()
    if hasattr(lib, "vp8g_k3_hang") and lib.vp8g_k3_hang(hang):
        import collections
        import numpy as np  # noqa: E402
        hr = np.ctypeslib.as_array(hang).reshape(1024, 4, 10)
        recs = collections.Counter()
        for b in range(min(B, 1024)):
            for w in range(4):
                r = hr[b, w]
                if r[7] & 0x80000000:
                    site = int(r[0])
                    poff = int(r[1])
                    what = ("rowdone[%d]" % ((poff - int(r[8])) // 4)) if site == 3 else \
                           ("fold_ptr" if poff == int(r[9]) else "off %d" % poff)
                    recs[(w, site, what, int(r[2]), int(r[3]), int(r[4]), int(np.int32(r[5])),
                          int(r[6]) & 3, int(r[7]) & 0xffff)] += 1
        print("K3_HANG (worker, site, word, waited-for, seen, y, x (neg: before waits), "
              "bar%4, G.abort): count")
        for k, v in recs.most_common(24):
            print("K3_HANG", k, v)
    if not hasattr(lib, "vp8g_k3_trace"):
        sys.exit(0)
fn = lib.vp8g_k3_trace
fn.restype = C.c_int
fn.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
NB = 1024
arr = (C.c_ulonglong * (NB * 4 * len(SLOTS)))()
nb = fn(arr, NB)
assert nb > 0, "not a K3_TRACE build"
import numpy as np  # noqa: E402
a = np.ctypeslib.as_array(arr).reshape(NB, 4, len(SLOTS)).astype(np.float64)
live = a[:, :, SLOTS.index("total")] > 0
wk = a[live]                     # (workers, slots)
tot = wk[:, SLOTS.index("total")].sum()
nmb = wk[:, SLOTS.index("n_mb")].sum()
res = {"workload": "%dx%d batch %d q%g m%d" % (W, H, B, quality, method),
       "k_encode_ms": round(t[6] / 1e3, 3), "workers": int(live.sum()), "mbs": int(nmb),
       "cycles_per_worker": round(tot / live.sum()), "share_of_worker_cycles": {},
       "cycles_per_mb": {}, "counts": {}}
for i, n in enumerate(SLOTS):
    v = wk[:, i].sum()
    if n.startswith("n_"):
        res["counts"][n] = int(v)
    else:
        res["share_of_worker_cycles"][n] = round(v / tot, 4)
        res["cycles_per_mb"][n] = round(v / max(nmb, 1))
# by worker index inside the workgroup (worker 0 leads rows 0, NW, ...)
res["per_worker_index"] = {}
for w in range(4):
    m = live[:, w]
    if m.any():
        x = a[m, w]
        T = x[:, SLOTS.index("total")].sum()
        res["per_worker_index"][w] = {n: round(x[:, i].sum() / T, 4) for i, n in enumerate(SLOTS)
                                      if not n.startswith("n_") and n != "total"}
print(json.dumps(res, indent=1))
if out_json:
    json.dump(res, open(out_json, "w"), indent=1)
