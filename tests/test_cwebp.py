"""cwebp links unchanged against libwebp_amd.so (caller
/root/reference/examples/cwebp.c:1122).

oracle/Makefile (target `$(OUT_REF)/cwebp`) compiles the reference's own
examples/cwebp.c and imageio/ readers against include/webp/encode.h and links
them with libwebp_amd.so for every encoder symbol, plus the reference's
decoder / demux / sharpyuv as the separate libraries libwebp ships them as (a
static archive without any src/enc object). The binary is test
infrastructure under oracle/_ref/ (git-ignored, travels to the GPU box).

CPU: the binary's encoder entry points are dynamic imports served by
libwebp_amd.so and no reference encoder code is inside it.
GPU: the unmodified CLI encodes syn-v1 PAM files to the SURVEY 8(d) known
answers (reference libwebp SHA-256s).
"""
import hashlib
import os
import subprocess

import pytest

from libwebp_amd.synth import syn_v1

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CWEBP = os.path.join(ROOT, "oracle", "_ref", "cwebp")
REF = "/root/reference/examples/cwebp.c"


def cwebp_binary():
    if os.path.exists(REF):   # dev container: (re)build it from the reference's sources
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "_ref/cwebp"],
                       check=True, capture_output=True)
    if not os.path.exists(CWEBP):
        pytest.skip("oracle/_ref/cwebp not built (needs /root/reference)")
    return CWEBP


def write_pam(path, img):
    h, w = img.shape[:2]
    with open(path, "wb") as fh:
        fh.write(b"P7\nWIDTH %d\nHEIGHT %d\nDEPTH 4\nMAXVAL 255\nTUPLTYPE RGB_ALPHA\nENDHDR\n"
                 % (w, h))
        fh.write(img.tobytes())


def test_cwebp_links_libwebp_amd():
    exe = cwebp_binary()
    dyn = subprocess.run(["readelf", "-d", exe], capture_output=True, text=True, check=True).stdout
    assert "[libwebp_amd.so]" in dyn
    und = subprocess.run(["nm", "-D", "--undefined-only", exe], capture_output=True, text=True,
                         check=True).stdout.split()
    for sym in ("WebPEncode", "WebPConfigInitInternal", "WebPPictureImportRGBA",
                "WebPPictureFree", "WebPMemoryWrite", "WebPPictureDistortion",
                "WebPGetEncoderVersion"):
        assert sym in und, sym
    # nothing of the reference encoder is linked into the binary
    syms = subprocess.run(["nm", exe], capture_output=True, text=True, check=True).stdout
    defined = {l.split()[-1] for l in syms.splitlines() if len(l.split()) == 3}
    for sym in ("WebPEncode", "VP8EncAnalyze", "VP8EncTokenLoop", "VP8EncWrite",
                "VP8LEncodeImage", "WebPPictureImportRGBA", "VP8Decimate"):
        assert sym not in defined, sym
    # the version query goes to libwebp_amd.so (no GPU needed)
    out = subprocess.run([exe, "-version"], capture_output=True, text=True, check=True).stdout
    assert out.splitlines()[0] == "1.3.2"


@pytest.mark.gpu
@pytest.mark.parametrize("w,h,f,args,sha", [
    (512, 512, 0, [], "48f759697c75eafe3b34a928b744faf118c233f017cf78445924127fe9ac5064"),
    (512, 512, 7, ["-q", "75", "-m", "4"],
     "60d5fba7e8bf7633f5852e6b5447a888ab1e4afa5cec65b1b53b7b9308f26a93"),
    (1920, 1080, 0, [], "8c12ebfcd2520d80829ae805673344fc2142b816116e3d2893ba93491378a185"),
])
def test_cwebp_cli_encodes_known_answers(gpu, tmp_path, w, h, f, args, sha):
    exe = CWEBP
    if not os.path.exists(exe):
        pytest.fail("oracle/_ref/cwebp missing: build it in the dev container (make -C oracle ref)")
    src, dst = str(tmp_path / "in.pam"), str(tmp_path / "out.webp")
    write_pam(src, syn_v1(w, h, f))
    r = subprocess.run([exe, "-quiet"] + args + [src, "-o", dst], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    with open(dst, "rb") as fh:
        assert hashlib.sha256(fh.read()).hexdigest() == sha
