"""Token partitions (cwebp -partitions N, config->partitions): VP8EncLoop
(methods 0-2, and methods 3-6 with low_memory) writes MB row y's tokens into
bit writer y & (2^partitions - 1) (src/enc/iterator_enc.c:48), each finished
on its own; VP8EncWrite puts the sizes of all partitions but the last after
partition 0 (src/enc/syntax_enc.c:248-265, 320-389) and partition 0 carries
log2 of the count (:283-285). The token loop (methods 3-6 without
low_memory) keeps a single partition (src/enc/webp_enc.c:115-122).

Parity: bit-exact bitstreams. Golden vectors from the reference build
(tests/golden/partitions_kat.json, make_options_golden.py); the oracle's
restatement is checked against them on CPU. On the GPU the compact token
stream's rows are regrouped per partition (k_partition) and K4 codes every
(frame, partition) stream; checked against the golden vectors through
WebPEncode and against the oracle from an HBM batch, including frames with
fewer MB rows than partitions (empty partitions).
"""
import hashlib
import json
import os

import numpy as np
import pytest

from libwebp_amd.synth import syn_v1

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CASES = [
    (64, 48, 0, {"quality": 75.0, "method": 0, "partitions": 1}),
    (128, 96, 1, {"quality": 30.0, "method": 1, "partitions": 2}),
    (333, 257, 2, {"quality": 90.0, "method": 2, "partitions": 3}),
    (17, 9, 3, {"quality": 50.0, "method": 2, "partitions": 3}),      # 1 MB row: 7 empty
    (40, 40, 4, {"quality": 75.0, "method": 0, "partitions": 2}),     # 3 rows over 4
    (200, 144, 4, {"quality": 99.0, "method": 1, "partitions": 2, "segments": 1}),
    (240, 160, 6, {"quality": 70.0, "method": 2, "partitions": 1, "autofilter": 1}),
    (96, 96, 7, {"quality": 0.0, "method": 0, "partitions": 3}),
    (333, 257, 2, {"quality": 75.0, "method": 3, "low_memory": 1, "partitions": 3}),
    (240, 160, 5, {"quality": 60.0, "method": 4, "low_memory": 1, "partitions": 2}),
    (128, 96, 1, {"quality": 80.0, "method": 6, "low_memory": 1, "partitions": 1}),
    (128, 96, 1, {"quality": 75.0, "method": 4, "partitions": 3}),     # token loop: one
    (1920, 1080, 0, {"quality": 75.0, "method": 2, "partitions": 3}),
    (1920, 1080, 1, {"quality": 75.0, "method": 4, "low_memory": 1, "partitions": 2}),
]


def kat():
    return json.load(open(os.path.join(ROOT, "tests", "golden", "partitions_kat.json")))["cases"]


def sha(b):
    return hashlib.sha256(b).hexdigest()


def test_golden_inputs_pinned():
    k = kat()
    assert len(k) == len(CASES)
    for (w, h, f, kw), c in zip(CASES, k):
        assert (c["w"], c["h"], c["frame"], c["params"]) == (w, h, f, kw)
        assert sha(syn_v1(w, h, f).tobytes())[:16] == c["in_sha"]


@pytest.mark.parametrize("i", [i for i, c in enumerate(CASES) if c[0] * c[1] < 1000000])
def test_oracle_matches_reference(i):
    from oracle import oracle
    w, h, f, kw = CASES[i]
    assert sha(oracle.encode_rgba(syn_v1(w, h, f), **kw)) == kat()[i]["sha256"]


def test_oracle_partitions_decode():
    """The own decoder reads every partition layout back to the picture the
    single-partition stream gives (the partitions only regroup the tokens)."""
    from oracle import oracle
    img = syn_v1(96, 80, 3)
    ref = oracle.decode_rgba(oracle.encode_rgba(img, quality=70.0, method=1))
    for p in (1, 2, 3):
        out = oracle.encode_rgba(img, quality=70.0, method=1, partitions=p)
        assert np.array_equal(oracle.decode_rgba(out), ref), p


@pytest.mark.gpu
def test_gpu_webpencode_partitions(gpu):
    for (w, h, f, kw), c in zip(CASES, kat()):
        out = gpu.encode_rgba(syn_v1(w, h, f), **kw)
        assert (len(out), sha(out)) == (c["size"], c["sha256"]), (w, h, f, kw)


@pytest.mark.gpu
def test_gpu_batch_partitions(gpu):
    import torch
    from oracle import oracle
    w, h, n = 176, 144, 4
    frames = np.stack([syn_v1(w, h, f) for f in range(n)])
    buf = torch.from_numpy(frames).to("cuda:0")
    torch.cuda.synchronize()
    for kw in ({"quality": 65.0, "method": 0, "partitions": 3},
               {"quality": 65.0, "method": 2, "partitions": 1},
               {"quality": 65.0, "method": 5, "low_memory": 1, "partitions": 2}):
        enc = gpu.GpuBatch(w, h, n, **kw)
        enc.encode_device(buf.data_ptr(), n)
        for f in range(n):
            assert enc.output(f) == oracle.encode_rgba(frames[f], **kw), (kw, f)
        enc.close()
