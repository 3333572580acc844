"""Parity of the HIP path (through the C-ABI of libwebp_amd.so) with the
reference: bit-exact YUV planes and bit-exact .webp bitstreams against the
golden vectors generated from the reference build, and against the oracle."""
import hashlib
import os

import numpy as np
import pytest

from libwebp_amd.synth import syn_v1

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def sha(b):
    return hashlib.sha256(b).hexdigest()


def test_import_planes_bit_exact(gpu, kat):
    for c in kat["import"]:
        enc = gpu.GpuBatch(c["w"], c["h"], 1)
        enc.encode_host(syn_v1(c["w"], c["h"], c["frame"])[None])
        y, u, v = enc.yuv(0)
        assert sha(np.ascontiguousarray(y).tobytes()) == c["y"], c
        assert sha(np.ascontiguousarray(u).tobytes()) == c["u"], c
        assert sha(np.ascontiguousarray(v).tobytes()) == c["v"], c
        enc.close()


def test_committed_bitstreams(gpu, kat):
    for name, digest in kat["bitstreams"].items():
        w, h = [int(t) for t in name.split("_")[1].split("x")]
        f = int(name.split("_f")[1].split("_")[0])
        enc = gpu.GpuBatch(w, h, 1)
        enc.encode_host(syn_v1(w, h, f)[None])
        assert sha(enc.output(0)) == digest, name
        enc.close()


def test_survey_kat_512_batch(gpu, kat):
    cases = [c for c in kat["survey"] if c["w"] == 512]
    frames = np.stack([syn_v1(512, 512, c["frame"]) for c in cases])
    enc = gpu.GpuBatch(512, 512, len(cases))
    enc.encode_host(frames)
    for i, c in enumerate(cases):
        out = enc.output(i)
        assert len(out) == c["size"] and sha(out) == c["sha256"], c["frame"]
    enc.close()


def test_survey_kat_1080p_hbm_batch(gpu, kat):
    """8 frames generated in HBM (syn-v1), encoded as one device-resident batch."""
    import torch
    cases = [c for c in kat["survey"] if c["w"] == 1920]
    n = len(cases)
    buf = torch.empty(n * 1920 * 1080 * 4, dtype=torch.uint8, device="cuda")
    gpu.synth_device(buf.data_ptr(), 1920, 1080, 0, n)
    torch.cuda.synchronize()
    enc = gpu.GpuBatch(1920, 1080, n)
    enc.encode_device(buf.data_ptr(), n)
    for i, c in enumerate(cases):
        assert c["frame"] == i
        out = enc.output(i)
        assert len(out) == c["size"] and sha(out) == c["sha256"], i
    enc.close()


def _sweep_params():
    import json
    k = json.load(open(os.path.join(HERE, "golden", "kat.json")))
    return [pytest.param(c, id="%dx%d_f%d_m%d_q%g" % (c["w"], c["h"], c["frame"], c["params"]["method"],
                                                     c["params"]["quality"]))
            for c in k["sweep"]]


@pytest.mark.parametrize("case", _sweep_params())
def test_sweep_configs(gpu, case):
    c = case
    enc = gpu.GpuBatch(c["w"], c["h"], 1, **c["params"])
    enc.encode_host(syn_v1(c["w"], c["h"], c["frame"])[None])
    out = enc.output(0)
    enc.close()
    assert sha(out) == c["sha256"]


def test_webpencode_single_picture_api(gpu, kat):
    """WebPPictureImportRGBA + WebPEncode (the drop-in entry points)."""
    for name, digest in kat["bitstreams"].items():
        w, h = [int(t) for t in name.split("_")[1].split("x")]
        f = int(name.split("_f")[1].split("_")[0])
        data, st = gpu.encode_rgba(syn_v1(w, h, f), stats=True)
        assert sha(data) == digest
        assert st.coded_size == len(data)


def test_oracle_random_small(gpu):
    from oracle import oracle
    rnd = np.random.RandomState(5)
    for _ in range(12):
        w, h = int(rnd.randint(1, 90)), int(rnd.randint(1, 90))
        q = float(rnd.randint(0, 101))
        img = syn_v1(w, h, int(rnd.randint(0, 1000)))
        enc = gpu.GpuBatch(w, h, 1, quality=q, method=4)
        enc.encode_host(img[None])
        assert enc.output(0) == oracle.encode_rgba(img, quality=q, method=4), (w, h, q)
        enc.close()


def test_transparent_input_gets_alph_chunk(gpu):
    """One translucent pixel: VP8X + ALPH + VP8 (tests/test_alpha.py has the
    parity checks), also with alpha level reduction (alpha_quality < 100)."""
    img = syn_v1(32, 32, 0).copy()
    img[5, 5, 3] = 10
    enc = gpu.GpuBatch(32, 32, 1)
    enc.encode_host(img[None])
    assert enc.error(0) == 0
    assert enc.output(0)[12:16] == b"VP8X"
    enc.close()
    enc = gpu.GpuBatch(32, 32, 1, alpha_quality=90)
    enc.encode_host(img[None])
    assert enc.error(0) == 0
    assert enc.output(0)[12:16] == b"VP8X"
    enc.close()


def test_survey_kat_4096_q90_m6(gpu, kat):
    """Config 4: one 4096x4096 frame at q90 m6 (trellis on
    every block), bit-exact against the reference's known answer."""
    (c,) = [c for c in kat["survey"] if c["w"] == 4096]
    enc = gpu.GpuBatch(4096, 4096, 1, **c["params"])
    enc.encode_host(syn_v1(4096, 4096, c["frame"])[None])
    out = enc.output(0)
    st = enc.timings()
    enc.close()
    assert len(out) == c["size"] and sha(out) == c["sha256"]
    print("4096x4096 q90 m6: k_encode %.0f ms" % (st[6] / 1e3))


def test_p0_overflow_rerun(gpu, kat):
    """Partition-0 overflow retry on the GPU (K3 pass_mode 1): a 5120x5120
    syn-v1 frame at q95 m4 needs 3 passes; the bitstream equals the
    reference's."""
    import torch
    (c,) = kat["p0_overflow"]
    w, h = c["w"], c["h"]
    buf = torch.empty(w * h * 4, dtype=torch.uint8, device="cuda")
    gpu.synth_device(buf.data_ptr(), w, h, c["frame"], 1)
    torch.cuda.synchronize()
    enc = gpu.GpuBatch(w, h, 1, **c["params"])
    enc.encode_device(buf.data_ptr(), 1)
    out = enc.output(0)
    err = enc.error(0)
    enc.close()
    assert err == 0
    assert len(out) == c["size"] and sha(out) == c["sha256"]


def _decode_kat():
    import json
    return json.load(open(os.path.join(HERE, "golden", "decode_kat.json")))["cases"]


def test_gpu_decode_equivalence(gpu):
    """north_star's criterion: the GPU bitstreams decode (own decoder,
    oracle/webp_dec.c) to the reference decoder's pixels for the reference
    encoder's bitstreams -- committed decoded-pixel hashes, YUV and RGBA."""
    import torch
    from oracle import oracle
    for c in _decode_kat():
        w, h, f = c["w"], c["h"], c["frame"]
        buf = torch.empty(w * h * 4, dtype=torch.uint8, device="cuda")
        gpu.synth_device(buf.data_ptr(), w, h, f, 1)
        torch.cuda.synchronize()
        enc = gpu.GpuBatch(w, h, 1, quality=c["q"], method=c["m"])
        enc.encode_device(buf.data_ptr(), 1)
        data = enc.output(0)
        enc.close()
        y, u, v = oracle.decode_yuv(data)
        assert sha(y.tobytes() + u.tobytes() + v.tobytes()) == c["yuv_sha256"], (w, h, f)
        assert sha(oracle.decode_rgba(data).tobytes()) == c["rgba_sha256"], (w, h, f)
