# CPU emulation of k_vp8l_dp + k_vp8l_dpwalk (LDS tile indexing, row wrap, sorted candidates,
# two cost rounds) against oracle vp8l_model.dp_parse; a design check run on the CPU.
import sys
import os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, 'tests'))
import numpy as np
from oracle import vp8l_model as M
from test_vp8l import lossless_picture, quantized

HASH_MUL = 0x1e35a7bd
def prefix(v):
    s, nb, _ = M.prefix_encode(v); return s, nb

def gpu_dp(argb, minb, cb, costs_np, dpcand):
    H, W = argb.shape
    E = argb.ravel().astype(np.int64)
    G, R, B, A, D = costs_np
    NG = 280 + 512
    cost = np.zeros(NG + 3 * 256 + 40, np.int64)
    cost[:len(G)] = G; cost[NG:NG+256] = R; cost[NG+256:NG+512] = B; cost[NG+512:NG+768] = A; cost[NG+768:NG+768+len(D)] = D
    oR, oB, oA, oD = NG, NG + 256, NG + 512, NG + 768
    nc = len(dpcand)
    lcost = [0] * 65
    for k in range(1, 65):
        s, nb = prefix(k); lcost[k] = cost[256 + s] + 256 * nb
    dcost = []
    for (d, dy, dx, code) in dpcand:
        s, nb = prefix(code); dcost.append(cost[oD + s] + 256 * nb)
    order = sorted(range(nc), key=lambda c: (dcost[c], c))
    choice = np.zeros(H * W, np.int64)
    for r0 in range(0, H, 64):
        runs = np.zeros((nc, 64), np.int64)
        ring = np.zeros((64, 66), np.int64)
        for ln in range(64): ring[ln][W % 65] = 0
        trow0 = r0 - 9
        c0 = ((W - 1) >> 6) << 6
        while c0 >= 0:
            tcol0 = c0 - 8
            tile = np.zeros((73, 80), np.int64)
            for tr in range(73):
                for tc in range(80):
                    rr, cc = trow0 + tr, tcol0 + tc
                    tile[tr][tc] = E[rr * W + cc] if (0 <= rr < H and 0 <= cc < W) else 0
            jt = min(63, W - 1 - c0)
            for jj in range(jt, -1, -1):
                j = c0 + jj
                for ln in range(64):
                    r = r0 + ln
                    if r >= H: continue
                    e = tile[ln + 9][jj + 8]
                    for c in range(nc):
                        d, dy, dx, code = dpcand[c]
                        sc, sr = j - dx, r - dy
                        if sc < 0: sc += W; sr -= 1
                        elif sc >= W: sc -= W; sr += 1
                        eq = False
                        if sr >= 0:
                            tr, tc = sr - trow0, sc - tcol0
                            if tr >= 0 and 0 <= tc < 80: eq = tile[tr][tc] == e
                            else: eq = E[sr * W + sc] == e
                        runs[c][ln] = min(runs[c][ln] + 1, 64) if eq else 0
                    m = minb[r * W + j]
                    if cb > 0 and m <= cb:
                        lit = cost[280 + (((int(e) * HASH_MUL) & 0xffffffff) >> (32 - cb))] * 68 // 100
                    else:
                        lit = (cost[(e >> 8) & 255] + cost[oR + ((e >> 16) & 255)] + cost[oB + (e & 255)] + cost[oA + (e >> 24)]) * 82 // 100
                    best = ring[ln][(j + 1) % 65] + lit; bk, bc = 1, 0
                    kmax = min(64, W - j); maxl = 1
                    for i in range(nc):
                        c = order[i]; L = min(runs[c][ln], kmax)
                        if L <= maxl: continue
                        for k in range(maxl + 1, L + 1):
                            v = ring[ln][(j + k) % 65] + dcost[c] + lcost[k]
                            if v < best: best, bk, bc = v, k, c
                        maxl = L
                    ring[ln][j % 65] = best
                    choice[r * W + j] = bk | (bc << 7)
            c0 -= 64
    # walk
    act = np.zeros(H * W, np.int64); clen = np.zeros(H * W, np.int64); ccode = np.zeros(H * W, np.int64)
    for r in range(H):
        x = 0
        while x < W:
            q = r * W + x; w = choice[q]; k = w & 127
            if k >= 2:
                act[q] = 2; clen[q] = k; ccode[q] = dpcand[(w >> 7) & 31][3]; act[q+1:q+k] = 3; x += k
            else:
                act[q] = 1 if (cb > 0 and minb[q] <= cb) else 0; x += 1
    return act.reshape(H, W), clen.reshape(H, W), ccode.reshape(H, W)

def cands(W):
    out = []
    for d in M.dp_candidates(W):
        dy = (d + W // 2) // W
        out.append((d, dy, d - dy * W, M.distance_code(W, d)))
    return out

for kind, w, h, f in [("q7", 80, 60, 0), ("q4", 37, 70, 1), ("q7", 9, 130, 3), ("q7", 200, 7, 2), ("q7", 1, 20, 1)]:
    img = quantized(w, h, int(kind[1:]), f)
    argb = M.to_argb(img)
    flat = argb.ravel()
    minb = M.cache_minb(flat)
    dists = M.candidate_distances(w)
    lens = M.match_lengths(argb, dists)
    act0, clen0, _ = M.parse(argb, (minb <= M.MAX_CACHE_BITS).reshape(h, w), dists, lens)
    cb = M.choose_cache_bits(argb, act0, clen0, minb.reshape(h, w))
    hit = (minb <= cb).reshape(h, w) if cb else np.zeros((h, w), bool)
    act, clen, ccode = M.parse(argb, hit, dists, lens)
    want = M.dp_parse(argb, hit, cb, act, clen, ccode)
    # GPU emulation: two rounds with costs from the previous parse
    a, l, c = act, clen, ccode
    for _ in range(2):
        (Gc, Rc, Bc, Ac, Dc), keys = M.dp_costs(argb, a, l, c, cb)
        a, l, c = gpu_dp(argb, minb, cb, (Gc, Rc, Bc, Ac, Dc), cands(w))
    ok = all(np.array_equal(x, y) for x, y in zip((a, l, c), want))
    print(kind, w, h, f, 'cb', cb, 'match' if ok else 'MISMATCH', int((a == 2).sum()))
