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


def window_coder(toks, seg, wd=32, stats=None, thr=7):
    """E1-E5 with E3 as k_emit_seg runs it: one forward pass per segment that
    places c_i most significant first through a 2*wd-bit window sliding down
    wd bits at a time, staged words, carries out of the window rippling into
    the words already written, the top-straddling word held back and the bits
    above the segment's top in H (added by E4). The upper word is staged once
    p - B <= thr (the kernel: wd=32, thr=7, so >= 17 bits of headroom above
    the current byte); a small wd or a large thr makes the carry path
    frequent."""
    n = len(toks)
    nseg = (n + seg - 1) // seg
    mask = (1 << wd) - 1
    assert 7 <= thr <= wd - 8         # p stays >= B; the upper word gets no direct adds
    r, cum, starts = 254, 0, []
    for s in range(nseg):             # E1/E2: true start ranges and shift counts
        starts.append((r, cum))
        for b, p in toks[s * seg:(s + 1) * seg]:
            r, _, k = _step(r, b, p)
            cum += k
    t = cum - 8
    nb = t if t <= 0 else t - 8 * ((t + 7) // 8)
    spad = 0
    for _ in range(9 - nb):
        r, _, k = _step(r, 0, 128)
        spad += k
    S = cum + spad
    L = (S + 7) // 8
    W = {}
    Hs = []
    for s in range(nseg):
        r, before = starts[s]
        part = toks[s * seg:(s + 1) * seg]
        segS = sum(_step_chain(r, part))
        top = S - before
        T = top - segS
        o = {"topw": 0, "H": 0}

        def put(wp, v):
            if not v:
                return
            assert wp >= 0
            if wp + wd <= top:
                if wp >= T:
                    assert W.get(wp // wd, 0) == 0
                    W[wp // wd] = v
                else:
                    W[wp // wd] = W.get(wp // wd, 0) | v
            elif wp < top:
                k = top - wp
                o["topw"] += v & ((1 << k) - 1)
                o["H"] += v >> k
            else:
                o["H"] += v << (wp - top)

        def carry(q):
            if stats is not None:
                stats["carries"] = stats.get("carries", 0) + 1
            while True:
                wp = q - q % wd
                if q >= top:
                    o["H"] += 1 << (q - top)
                    return
                if wp + wd > top:
                    k = top - wp
                    o["topw"] += 1 << (q - wp)
                    if o["topw"] >> k:
                        o["topw"] -= 1 << k
                        o["H"] += 1
                    return
                old = W.get(wp // wd, 0)
                W[wp // wd] = (old + (1 << (q - wp))) & mask
                if old + (1 << (q - wp)) <= mask:
                    return
                q = wp + wd

        p = top
        B = (top - thr) - (top - thr) % wd   # top - B in [thr, thr + wd)
        acc, stg = 0, []
        for b, pr in part:
            r, c, k = _step(r, b, pr)
            assert 0 <= p - B <= thr + wd
            na = acc + (c << (p - B))
            if na >> (2 * wd):
                for i, v in enumerate(stg):
                    put(B + 2 * wd + wd * (len(stg) - 1 - i), v)
                stg = []
                carry(B + 2 * wd)
                na &= (1 << (2 * wd)) - 1
            acc = na
            p -= k
            if p - B <= thr:
                stg.append(acc >> wd)
                acc = (acc & mask) << wd
                B -= wd
        assert p == T
        for i, v in enumerate(stg):
            put(B + 2 * wd + wd * (len(stg) - 1 - i), v)
        put(B + wd, acc >> wd)
        put(B, acc & mask)
        if top % wd and o["topw"]:
            W[top // wd] = W.get(top // wd, 0) | o["topw"]
        assert o["H"] < 256
        Hs.append((top, o["H"]))
    N = sum(v << (wd * i) for i, v in W.items())
    for top, h in Hs:                 # E4: H_s added at the segment's top
        N += h << top
    return (N >> 1).to_bytes(L, "big") if L else b""


def _step_chain(r, part):
    for b, p in part:
        r, _, k = _step(r, b, p)
        yield k


def _carry_heavy(rng, n):
    """Long runs of 1 bits push the coder's low end towards the top of its
    interval: all-ones words, then carries."""
    toks = []
    while len(toks) < n:
        if rng.random() < 0.5:
            p = rng.choice([128, 200, 250, 16])
            toks.extend([(1, p)] * rng.randint(5, 120))
        else:
            for _ in range(rng.randint(1, 20)):
                p = rng.randint(1, 255)
                toks.append((rng.randint(0, 1), p))
    return toks[:n]


def _carry_forcing(rng, n):
    """Streams that make the coder's low end run up to a point from below (a
    long run of 1 bits in N) and then cross it (a carry through the whole
    run): each episode takes the midpoint of the current interval and codes
    the bits whose subintervals hold a point just below it, then just above
    it; random tokens in between. Exact interval arithmetic (A / 2^M)."""
    M = 8 * n + 64
    st = {"A": 0, "r": 254, "P": 0}
    toks = []

    def put(b, p):
        r = st["r"]
        split = (r * p) >> 8
        if b:
            st["A"] += (split + 1) << (M - st["P"])
            r = r - split - 1
        else:
            r = split
        sh = 0
        while ((r + 1) << sh) < 128:
            sh += 1
        st["r"] = ((r + 1) << sh) - 1
        st["P"] += sh
        toks.append((b, p))

    while len(toks) < n:
        if rng.random() < 0.3:
            for _ in range(rng.randint(1, 30)):
                put(rng.randint(0, 1), rng.randint(1, 255))
            continue
        mid = st["A"] + ((st["r"] + 1) << (M - st["P"] - 1))
        eps = 1 << max(0, M - st["P"] - 90)
        for target, k in ((mid - eps, rng.randint(30, 80)), (mid + eps, rng.randint(20, 80))):
            for _ in range(k):
                if len(toks) >= n or st["P"] + 8 >= M - 64:
                    break
                p = rng.choice([128, 100, 160, 200, 60])
                bound = st["A"] + ((((st["r"] * p) >> 8) + 1) << (M - st["P"]))
                put(0 if target < bound else 1, p)
    return toks[:n]


def test_window_pass_matches_reference_coder():
    rng = random.Random(11)
    st16, st32 = {}, {}
    for it in range(120):
        n = rng.randint(0, 3000)
        if it % 2:
            toks = _carry_heavy(rng, n)
        else:
            toks = []
            for _ in range(n):
                p = rng.randint(1, 255)
                toks.append((1 if rng.random() * 256 >= p else 0, p))
        seg = rng.choice([1, 3, 64, 200, 2048])
        want = ref_coder(toks)
        assert window_coder(toks, seg, 32, st32) == want
        assert window_coder(toks, seg, 32, None, 24) == want
        assert window_coder(toks, seg, 15, st16) == want
    assert st16.get("carries", 0) > 20   # the carry path ran
    st = {}
    for _ in range(4):   # and with the kernel's own window
        toks = _carry_forcing(rng, 5000)
        assert window_coder(toks, rng.choice([64, 2048]), 32, st) == ref_coder(toks)
    assert st.get("carries", 0) > 20
