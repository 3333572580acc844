"""The segmented boolean-coder model behind K4 (hip/vp8_emit.hip), checked
on CPU against a direct restatement of libwebp's VP8PutBit / Flush /
VP8BitWriterFinish (src/utils/bit_writer_utils.c:55-124,199-206) on random
(bit, probability) streams: the output is the big-endian bytes of N >> 1
on L = (S + 7) / 8 bytes, N = sum c_i 2^E_i, and cutting the stream into
segments whose start ranges come from per-segment range maps reproduces it."""
import random


def ref_coder(toks):
    """bit_writer_utils.c: VP8PutBit + Flush + VP8BitWriterFinish."""
    st = {"range": 254, "value": 0, "nb": -8, "run": 0}
    buf = []

    def flush():
        s = 8 + st["nb"]
        bits = st["value"] >> s
        st["value"] -= bits << s
        st["nb"] -= 8
        if (bits & 0xff) != 0xff:
            if bits & 0x100 and buf:
                buf[-1] += 1
            buf.extend([0x00 if bits & 0x100 else 0xff] * st["run"])
            st["run"] = 0
            buf.append(bits & 0xff)
        else:
            st["run"] += 1

    def put(bit, p):
        split = (st["range"] * p) >> 8
        if bit:
            st["value"] += split + 1
            st["range"] -= split + 1
        else:
            st["range"] = split
        if st["range"] < 127:
            sh = 0
            while ((st["range"] + 1) << sh) < 128:
                sh += 1
            st["range"] = ((st["range"] + 1) << sh) - 1
            st["value"] <<= sh
            st["nb"] += sh
            if st["nb"] > 0:
                flush()

    for b, p in toks:
        put(b, p)
    for _ in range(9 - st["nb"]):
        put(0, 128)
    st["nb"] = 0
    flush()
    return bytes(buf)


def _step(r, b, p):
    split = (r * p) >> 8
    c = split + 1 if b else 0
    r = r - split - 1 if b else split
    sh = 0
    while ((r + 1) << sh) < 128:
        sh += 1
    return ((r + 1) << sh) - 1, c, sh


def seg_coder(toks, seg):
    """E1-E5 of vp8_emit.hip in exact integer arithmetic."""
    n = len(toks)
    nseg = (n + seg - 1) // seg
    maps = []
    for s in range(nseg):
        part = toks[s * seg:(s + 1) * seg]
        m = []
        for r0 in range(127, 255):
            r, tot = r0, 0
            for b, p in part:
                r, _, k = _step(r, b, p)
                tot += k
            m.append((r, tot))
        maps.append(m)
    r, cum, starts = 254, 0, []
    for s in range(nseg):
        starts.append((r, cum))
        r, k = maps[s][r - 127]
        cum += k
    t = cum - 8
    nb = t if t <= 0 else t - 8 * ((t + 7) // 8)
    spad = 0
    for _ in range(9 - nb):
        r, _, k = _step(r, 0, 128)
        spad += k
    S = cum + spad
    L = (S + 7) // 8
    N = 0
    for s in range(nseg):
        r, before = starts[s]
        cs = []
        for b, p in toks[s * seg:(s + 1) * seg]:
            r, c, k = _step(r, b, p)
            cs.append((c, k))
        E, P = 0, 0
        for c, k in reversed(cs):
            E += k
            P += c << E
        N += P << (S - (before + E))
    return (N >> 1).to_bytes(L, "big") if L else b""


def test_segmented_model_matches_reference_coder():
    rng = random.Random(3)
    for _ in range(150):
        n = rng.randint(0, 1500)
        toks = []
        for _ in range(n):
            p = rng.randint(1, 255)
            b = 1 if rng.random() * 256 >= p else 0
            if rng.random() < 0.05:
                b = rng.randint(0, 1)
            toks.append((b, p))
        seg = rng.choice([1, 3, 64, 200, 2048])
        assert seg_coder(toks, seg) == ref_coder(toks)
