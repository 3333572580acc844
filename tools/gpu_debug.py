"""Stage-by-stage GPU vs oracle comparison (debug aid, runs on the GPU box)."""
import hashlib
import sys
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import libwebp_amd
from libwebp_amd.synth import syn_v1
from oracle import oracle


def compare(w, h, f=0, **kw):
    img = syn_v1(w, h, f)
    enc = libwebp_amd.GpuBatch(w, h, 1, **kw)
    enc.encode_host(img[None])
    y, u, v = enc.yuv(0)
    oy, ou, ov = oracle.import_rgba(img)
    imp_ok = (y == oy).all() and (u == ou).all() and (v == ov).all()
    ref, tr = oracle.encode_yuv(oy, ou, ov, trace=True, **kw)
    err = enc.error(0)
    out = enc.output(0) if err == 0 else b""
    same = out == ref
    print("%dx%d f%d %s import_ok=%s err=%d size gpu=%d ref=%d %s" % (
        w, h, f, kw, imp_ok, err, len(out), len(ref), "OK" if same else "MISMATCH"))
    if not same:
        info = enc.mbinfo(0)
        nbad = 0
        for i, t in enumerate(tr):
            g = info[i]
            om = (t.type, t.uv_mode, t.segment, t.skip) + tuple(t.modes)
            gm = tuple(int(x) for x in g)
            if om != gm:
                print("  MB %d (x=%d,y=%d): oracle %s gpu %s" % (
                    i, i % ((w + 15) // 16), i // ((w + 15) // 16), om, gm))
                nbad += 1
                if nbad > 5:
                    break
        if nbad == 0:
            print("  all MB decisions equal; diff is in tokens/probas/headers")
    print("  timings", ["%.0f" % t for t in enc.timings()])
    enc.close()
    return same


if __name__ == "__main__":
    print("devices", libwebp_amd.device_count())
    ok = True
    for (w, h) in [(16, 16), (64, 48), (33, 17), (128, 128), (333, 257), (512, 512)]:
        ok &= compare(w, h)
    for m in (3, 5, 6):
        for (w, h) in [(64, 48), (128, 128)]:
            ok &= compare(w, h, method=m)
    ok &= compare(256, 256, quality=90, method=6)
    sys.exit(0 if ok else 1)
