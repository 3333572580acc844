"""Size of every lossless fixture (tests/golden/lossless_kat.json) encoded on
the GPU against the reference encoder's size, one line per case plus the
worst ratio per kind (every kind within 3%).

usage: python tools/lossless_ratios.py [json_out [dump_dir]]
(dump_dir: every encoded file, <kind>_<w>x<h>_f<frame>.webp, for
oracle-side analysis)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import libwebp_amd as gpu  # noqa: E402
from test_vp8l import gpu_encode, lossless_cases, lossless_picture  # noqa: E402

out = sys.argv[1] if len(sys.argv) > 1 else None
dump = sys.argv[2] if len(sys.argv) > 2 else None
if dump:
    os.makedirs(dump, exist_ok=True)
rows, worst = [], {}
for c in lossless_cases(1 << 30):
    img = lossless_picture(c["kind"], c["w"], c["h"], c["frame"])
    data = gpu_encode(gpu, img[None])[0]
    got = len(data)
    if dump:
        open(os.path.join(dump, "%s_%dx%d_f%d.webp" % (c["kind"], c["w"], c["h"], c["frame"])),
             "wb").write(data)
    r = got / c["size"]
    rows.append({"kind": c["kind"], "w": c["w"], "h": c["h"], "frame": c["frame"],
                 "reference": c["size"], "ours": got, "ratio": round(r, 4)})
    k = c["kind"].rstrip("0123456789") or c["kind"]
    worst[k] = max(worst.get(k, 0.0), round(r, 4))
    print("%-7s %5dx%-5d f%d  ref %9d  ours %9d  %.4f" % (c["kind"], c["w"], c["h"], c["frame"],
                                                          c["size"], got, r), flush=True)
print("worst per kind:", json.dumps(worst))
if out:
    json.dump({"cases": rows, "worst_per_kind": worst}, open(out, "w"), indent=1)
