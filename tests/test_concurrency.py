"""Concurrent WebPEncode callers (SURVEY.md 8(b) threading row: the reference
is re-entrant for distinct pictures, src/enc/webp_enc.c:330-410). Each call
takes its own engine from the process-wide pool (host/webp_api.c) and runs on
its own HIP stream; K3X launches of the callers share one workgroup budget.
Outputs stay bit-exact (SURVEY 8(d) KATs) and the callers overlap on the GPU."""
import hashlib
import threading
import time

import numpy as np
import pytest

from libwebp_amd.synth import syn_v1

pytestmark = pytest.mark.gpu


def _encode_all(gpu, frames, nthreads):
    out = [None] * len(frames)
    errs = []

    def work(i0):
        try:
            for i in range(i0, len(frames), nthreads):
                out[i] = gpu.encode_rgba(frames[i], quality=75.0, method=4)
        except Exception as e:   # surfaced by the assert below
            errs.append(e)

    ts = [threading.Thread(target=work, args=(k,)) for k in range(nthreads)]
    t0 = time.perf_counter()
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    el = time.perf_counter() - t0
    assert not errs, errs
    return out, el


def test_threads_bit_exact_1080p(gpu, kat):
    cases = sorted((c for c in kat["survey"] if c["w"] == 1920), key=lambda c: c["frame"])
    frames = [syn_v1(1920, 1080, c["frame"]) for c in cases]
    gpu.encode_rgba(frames[0])   # engine creation outside the timed calls
    out, _ = _encode_all(gpu, frames, len(frames))
    for c, o in zip(cases, out):
        assert hashlib.sha256(o).hexdigest() == c["sha256"], c["frame"]


def test_threads_overlap(gpu, kat):
    """8 callers x 1080p frames: aggregate throughput above one caller's"""
    cases = sorted((c for c in kat["survey"] if c["w"] == 1920), key=lambda c: c["frame"])
    frames = [syn_v1(1920, 1080, c["frame"]) for c in cases] * 2
    _encode_all(gpu, frames[:8], 8)   # warm: one engine per caller
    _, t1 = _encode_all(gpu, frames, 1)
    out, t8 = _encode_all(gpu, frames, 8)
    want = {c["frame"]: c["sha256"] for c in cases}
    for i, o in enumerate(out):
        assert hashlib.sha256(o).hexdigest() == want[cases[i % 8]["frame"]]
    mps1 = len(frames) * 1920 * 1080 / t1 / 1e6
    mps8 = len(frames) * 1920 * 1080 / t8 / 1e6
    print("WebPEncode 1080p: 1 thread %.1f MP/s, 8 threads %.1f MP/s" % (mps1, mps8))
    assert mps8 > 1.5 * mps1, (mps1, mps8)


def test_threads_mixed_sizes(gpu, kat):
    """callers with different picture sizes share the pool without tearing
    engines down; small pictures check against the committed bitstreams"""
    sizes = [(512, 512, 0), (512, 512, 7), (1920, 1080, 1), (1920, 1080, 2)]
    want = {(c["w"], c["frame"]): c["sha256"] for c in kat["survey"]}
    frames = [syn_v1(w, h, f) for w, h, f in sizes] * 3
    out, _ = _encode_all(gpu, frames, 6)
    for i, o in enumerate(out):
        w, h, f = sizes[i % len(sizes)]
        assert hashlib.sha256(o).hexdigest() == want[(w, f)], (w, h, f)
