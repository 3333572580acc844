import sys, os, hashlib
sys.path.insert(0, os.getcwd())
import libwebp_amd
from libwebp_amd.synth import syn_v1
sys.path.insert(0, "tests")
import test_multipass as T
for (w, h, f, kw), c in zip(T.CASES, T.kat()):
    try:
        out = libwebp_amd.encode_rgba(syn_v1(w, h, f), **kw)
        ok = hashlib.sha256(out).hexdigest() == c["sha256"]
        print(w, h, f, kw, "ok" if ok else "MISMATCH", flush=True)
    except Exception as e:
        print(w, h, f, kw, "ERR", e, libwebp_amd.last_error(), flush=True)
