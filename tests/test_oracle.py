"""The oracle (oracle/vp8_oracle.c, CPU restatement) against the golden
vectors generated from the reference (tests/golden/make_golden.py) and, when
present, against the reference build itself."""
import hashlib
import random

import pytest

from libwebp_amd.synth import syn_v1
from oracle import oracle


def sha(b):
    return hashlib.sha256(b).hexdigest()


def test_synth_matches_survey_inputs(kat):
    for c in kat["survey"][:3] + kat["sweep"][:10]:
        if c["w"] * c["h"] > 2_500_000:
            continue
        assert sha(syn_v1(c["w"], c["h"], c["frame"]).tobytes())[:16] == c["in_sha"]


@pytest.mark.parametrize("idx", range(3))
def test_oracle_survey_kat(kat, idx):
    c = kat["survey"][idx]           # 512^2 f0, f7 and 1080p f0
    out = oracle.encode_rgba(syn_v1(c["w"], c["h"], c["frame"]), **c["params"])
    assert len(out) == c["size"]
    assert sha(out) == c["sha256"]


def test_oracle_sweep_kat(kat):
    bad = []
    for c in kat["sweep"]:
        out = oracle.encode_rgba(syn_v1(c["w"], c["h"], c["frame"]), **c["params"])
        if sha(out) != c["sha256"]:
            bad.append((c["w"], c["h"], c["frame"], c["params"]))
    assert not bad, bad


def test_oracle_import_planes(kat):
    for c in kat["import"]:
        y, u, v = oracle.import_rgba(syn_v1(c["w"], c["h"], c["frame"]))
        assert sha(y.tobytes()) == c["y"]
        assert sha(u.tobytes()) == c["u"]
        assert sha(v.tobytes()) == c["v"]


def test_oracle_committed_bitstreams(kat):
    import os
    here = os.path.join(os.path.dirname(__file__), "golden")
    for name, digest in kat["bitstreams"].items():
        data = open(os.path.join(here, name), "rb").read()
        assert sha(data) == digest
        w, h, f = [int(t) for t in name.split("_")[1].split("x")] + [int(name.split("_f")[1][0])]
        assert oracle.encode_rgba(syn_v1(w, h, f)) == data


def test_oracle_vs_reference_random(ref_lib):
    from libwebp_amd import abi
    rnd = random.Random(7)
    for _ in range(30):
        w, h = rnd.randint(1, 150), rnd.randint(1, 150)
        kw = dict(quality=float(rnd.randint(0, 100)), method=rnd.randint(3, 6),
                  segments=rnd.randint(1, 4), sns_strength=rnd.randint(0, 100),
                  filter_strength=rnd.randint(0, 100), filter_sharpness=rnd.randint(0, 7))
        img = syn_v1(w, h, rnd.randrange(100))
        ref, _ = abi.encode_rgba(ref_lib, img, **kw)
        assert oracle.encode_rgba(img, **kw) == ref, (w, h, kw)


def test_oracle_rejects_transparency():
    img = syn_v1(8, 8, 0).copy()
    img[3, 3, 3] = 7
    with pytest.raises(ValueError):
        oracle.import_rgba(img)


def test_oracle_p0_overflow_retry(kat):
    """Partition-0 overflow: the restatement re-runs the MB loop with a halved
    I4 header budget (frame_enc.c:869-876) and lands on the reference's
    bitstream (5120x5120 q95 m4: 3 passes)."""
    (c,) = kat["p0_overflow"]
    out = oracle.encode_rgba(syn_v1(c["w"], c["h"], c["frame"]), **c["params"])
    assert oracle.lib().vp8o_last_pass_count() == c["passes"] > 1
    assert len(out) == c["size"] and sha(out) == c["sha256"]
