"""Sharp (iterative) RGB->YUV import, use_sharp_yuv (SURVEY.md 8(a) row a12;
reference sharpyuv/sharpyuv.c:297-430 via picture_csp_enc.c:176-186).

CPU: the oracle restatement (oracle/sharp_oracle.c) against the golden
vectors generated from the reference build (tests/golden/make_golden.py
--only-sharp) and, when oracle/_ref is present, against the reference itself.
GPU: the HIP kernels (hip/vp8_sharp.hip) through the C-ABI against both."""
import hashlib

import numpy as np
import pytest

from libwebp_amd.synth import syn_v1
from oracle import oracle


def sha(b):
    return hashlib.sha256(b).hexdigest()


def planes_sha(y, u, v):
    return [sha(np.ascontiguousarray(p).tobytes()) for p in (y, u, v)]


def noise_200x130():
    img = np.random.RandomState(11).randint(0, 256, (130, 200, 4)).astype(np.uint8)
    img[..., 3] = 255
    return img


# ---------------------------------------------------------------- CPU (oracle)

def test_oracle_sharp_import_golden(kat):
    for c in kat["sharp"]["import"]:
        if c["w"] * c["h"] > 300_000:
            continue
        got = planes_sha(*oracle.import_rgba(syn_v1(c["w"], c["h"], c["frame"]), sharp=True))
        assert got == [c["y"], c["u"], c["v"]], c


def test_oracle_sharp_import_noise_golden(kat):
    want = kat["sharp"]["noise_200x130_seed11"]
    got = planes_sha(*oracle.import_rgba(noise_200x130(), sharp=True))
    assert got == [want["y"], want["u"], want["v"]]


def test_oracle_sharp_encode_golden(kat):
    for c in kat["sharp"]["encode"]:
        if c["w"] * c["h"] > 300_000:
            continue
        out = oracle.encode_rgba(syn_v1(c["w"], c["h"], c["frame"]), **c["params"])
        assert len(out) == c["size"] and sha(out) == c["sha256"], c


def test_sharp_differs_from_plain_import(kat):
    """The golden sharp planes are not the plain conversion (the test would
    otherwise not discriminate); tiny syn-v1 crops are flat tiles, where both
    agree."""
    plain = {(c["w"], c["h"], c["frame"]): c for c in kat["import"]}
    for c in kat["sharp"]["import"]:
        y, _, _ = oracle.import_rgba(syn_v1(c["w"], c["h"], c["frame"]))
        if 1000 <= c["w"] * c["h"] <= 300_000:
            assert sha(y.tobytes()) != c["y"], c
        p = plain.get((c["w"], c["h"], c["frame"]))
        if p:
            assert p["y"] != c["y"]


def test_oracle_sharp_vs_reference_random(ref_lib):
    from libwebp_amd import abi
    rnd = np.random.RandomState(21)
    for _ in range(12):
        w, h = int(rnd.randint(1, 90)), int(rnd.randint(1, 90))
        img = rnd.randint(0, 256, (h, w, 4)).astype(np.uint8) if rnd.rand() < 0.5 else \
            syn_v1(w, h, int(rnd.randint(0, 100)))
        img = np.ascontiguousarray(img)
        img[..., 3] = 255
        if w >= 4 and h >= 4:
            a = abi.picture_yuv(ref_lib, img, sharp=True)
            b = oracle.import_rgba(img, sharp=True)
            assert all(np.array_equal(x, y) for x, y in zip(a, b)), (w, h)
        q = float(rnd.randint(0, 101))
        ref, _ = abi.encode_rgba(ref_lib, img, quality=q, method=4, use_sharp_yuv=1)
        assert oracle.encode_rgba(img, quality=q, method=4, use_sharp_yuv=1) == ref, (w, h, q)


# ---------------------------------------------------------------- GPU (HIP)

@pytest.mark.gpu
def test_gpu_sharp_import_planes(gpu, kat):
    for c in kat["sharp"]["import"]:
        enc = gpu.GpuBatch(c["w"], c["h"], 1, use_sharp_yuv=1)
        enc.encode_host(syn_v1(c["w"], c["h"], c["frame"])[None])
        got = planes_sha(*enc.yuv(0))
        enc.close()
        assert got == [c["y"], c["u"], c["v"]], c


@pytest.mark.gpu
def test_gpu_sharp_import_noise(gpu, kat):
    want = kat["sharp"]["noise_200x130_seed11"]
    enc = gpu.GpuBatch(200, 130, 1, use_sharp_yuv=1)
    enc.encode_host(noise_200x130()[None])
    got = planes_sha(*enc.yuv(0))
    enc.close()
    assert got == [want["y"], want["u"], want["v"]]


@pytest.mark.gpu
def test_gpu_sharp_encode_golden(gpu, kat):
    for c in kat["sharp"]["encode"]:
        enc = gpu.GpuBatch(c["w"], c["h"], 1, **c["params"])
        enc.encode_host(syn_v1(c["w"], c["h"], c["frame"])[None])
        out = enc.output(0)
        enc.close()
        assert len(out) == c["size"] and sha(out) == c["sha256"], c


@pytest.mark.gpu
def test_gpu_sharp_hbm_batch_1080p(gpu, kat):
    """Two 1080p frames generated in HBM, one device-resident sharp batch."""
    import torch
    cases = [c for c in kat["sharp"]["encode"] if c["w"] == 1920]
    n = len(cases)
    buf = torch.empty(n * 1920 * 1080 * 4, dtype=torch.uint8, device="cuda")
    gpu.synth_device(buf.data_ptr(), 1920, 1080, 0, n)
    torch.cuda.synchronize()
    enc = gpu.GpuBatch(1920, 1080, n, **cases[0]["params"])
    enc.encode_device(buf.data_ptr(), n)
    for i, c in enumerate(cases):
        assert c["frame"] == i
        out = enc.output(i)
        assert len(out) == c["size"] and sha(out) == c["sha256"], i
    enc.close()


@pytest.mark.gpu
def test_gpu_sharp_webpencode_api(gpu, kat):
    """ARGB picture + WebPEncode(use_sharp_yuv=1): the cwebp -sharp_yuv path,
    and preprocessing & 4 (the older spelling of the same switch)."""
    for c in kat["sharp"]["encode"]:
        if c["w"] * c["h"] > 300_000:
            continue
        img = syn_v1(c["w"], c["h"], c["frame"])
        data = gpu.encode_rgba(img, **c["params"])
        assert sha(data) == c["sha256"], c
        p = dict(c["params"])
        p.pop("use_sharp_yuv")
        data = gpu.encode_rgba(img, use_argb=True, preprocessing=4, **p)
        assert sha(data) == c["sha256"], c


@pytest.mark.gpu
def test_gpu_sharp_random_vs_oracle(gpu):
    rnd = np.random.RandomState(8)
    for _ in range(10):
        w, h = int(rnd.randint(1, 120)), int(rnd.randint(1, 120))
        img = rnd.randint(0, 256, (h, w, 4)).astype(np.uint8)
        img[..., 3] = 255
        q = float(rnd.randint(0, 101))
        enc = gpu.GpuBatch(w, h, 1, quality=q, method=4, use_sharp_yuv=1)
        enc.encode_host(img[None])
        got = enc.output(0)
        yuv = enc.yuv(0)
        enc.close()
        want = oracle.import_rgba(img, sharp=True)
        assert all(np.array_equal(a, b) for a, b in zip(yuv, want)), (w, h)
        assert got == oracle.encode_rgba(img, quality=q, method=4, use_sharp_yuv=1), (w, h, q)
