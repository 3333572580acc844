"""The statistics fold's snapshot skip (DESIGN.md section 9, vp8_k3.hip
fold_mbs): a row's pending deltas stored every XS_SNAP_MBS MBs let the exact
replay of a saturating counter start at the last snapshot below its halving
point. This checks that rule against the reference's per-token update
(VP8RecordStats, src/enc/cost_enc.h:45-56: a counter whose count reaches
0xfffe is halved, rounding up, before the next bit is recorded) on random
token streams that cross the halving point zero, one or several times."""
import random

import pytest

SNAP = 16   # XS_SNAP_MBS


def record(p, bit):
    """VP8RecordStats on one packed counter (count << 16 | ones)"""
    if p >= 0xfffe0000:
        p = ((p + 1) >> 1) & 0x7fff7fff
    return p + 0x10000 + bit


def fold_reference(p, mbs):
    for bits in mbs:
        for b in bits:
            p = record(p, b)
    return p


def fold_with_snapshots(p, mbs, c0=0):
    """the kernel's fold of MBs [c0, len(mbs)) of a row: pending delta of the
    whole span, snapshots at the row's 16-MB boundaries inside the span
    (cumulative since c0), the last snapshot still below the halving point
    added at once, then the exact walk, then the rest added at once once no
    halving point is left"""
    span = mbs[c0:]
    n = sum(len(b) for b in span)
    k = sum(sum(b) for b in span)
    if (p >> 16) + n < 0xffff:          # no replay: one add
        return p + (n << 16) + k
    c1 = len(mbs)
    snaps = []                           # boundaries b in (c0, c1), lane order
    b = (c0 // SNAP + 1) * SNAP
    while b < c1 and len(snaps) < 64:
        cnt = sum(len(x) for x in mbs[c0:b])
        one = sum(sum(x) for x in mbs[c0:b])
        snaps.append((b, (cnt << 16) | one))
        b += SNAP
    ok = [(p >> 16) + (v >> 16) < 0xfffe for _, v in snaps]
    nok = sum(ok)
    assert ok == [True] * nok + [False] * (len(ok) - nok), "counts only grow: a prefix"
    start = c0
    if nok:
        bb, v = snaps[nok - 1]
        p += v
        n -= v >> 16
        k -= v & 0xffff
        start = bb
    for bits in mbs[start:]:
        if not n:
            break
        if (p >> 16) + n < 0xfffe:       # no halving point left in the row
            break
        for bit in bits:
            p = record(p, bit)
            n -= 1
            k -= bit
    return p + (n << 16) + k


def _row(rng, nmb, per_mb, p_one):
    return [[int(rng.random() < p_one) for _ in range(rng.randint(0, per_mb))]
            for _ in range(nmb)]


@pytest.mark.parametrize("seed", range(40))
def test_snapshot_skip_matches_record_stats(seed):
    rng = random.Random(seed)
    nmb = rng.choice([17, 120, 256])
    per_mb = rng.choice([30, 300, 3000])
    mbs = _row(rng, nmb, per_mb, rng.random())
    start = rng.choice([0, 0x8000, 0xff00, 0xfff0, 0xfffd, 0xfffe])
    p0 = (start << 16) | rng.randint(0, start)
    c0 = rng.choice([0, 0, rng.randrange(nmb)])
    assert fold_with_snapshots(p0, mbs, c0) == fold_reference(p0, mbs[c0:])


def test_several_halvings_in_one_row():
    rng = random.Random(7)
    mbs = _row(rng, 256, 3000, 0.3)      # ~384 K tokens: 5+ halvings from 0xfff0
    p0 = 0xfff0 << 16
    assert sum(len(b) for b in mbs) > 5 * 0x8000
    assert fold_with_snapshots(p0, mbs) == fold_reference(p0, mbs)
