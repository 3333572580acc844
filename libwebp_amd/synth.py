"""syn-v1 synthetic RGBA frames, vectorised in numpy.

Counter-based: every pixel is a pure function of (seed, frame, x, y), so any
frame can be generated independently (tests, bench, multi-rank sharding).
All arithmetic is uint64 with C wrap-around semantics.
"""
import numpy as np

_M = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix64(z):
    z = z + np.uint64(0x9E3779B97F4A7C15)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def syn_v1(width, height, frame=0, seed=1):
    """Return an (H, W, 4) uint8 RGBA array for frame `frame` of syn-v1."""
    with np.errstate(over="ignore"):
        y = np.arange(height, dtype=np.uint64)[:, None]
        x = np.arange(width, dtype=np.uint64)[None, :]
        key = (np.uint64(seed) << np.uint64(48)) ^ (np.uint64(frame) << np.uint64(32))
        h = _splitmix64(key ^ (y << np.uint64(16)) ^ x)
    xi = np.arange(width, dtype=np.int64)[None, :]
    yi = np.arange(height, dtype=np.int64)[:, None]
    region = ((xi >> 5) ^ (yi >> 5) ^ frame) & 3
    n = (h & np.uint64(31)).astype(np.int64) - 16
    gx = (xi * 255 // (width - 1)) if width > 1 else np.zeros_like(xi)
    gy = (yi * 255 // (height - 1)) if height > 1 else np.zeros_like(yi)
    shape = (height, width)
    r = np.empty(shape, np.int64)
    g = np.empty(shape, np.int64)
    b = np.empty(shape, np.int64)
    # region 0: flat tiles
    flat = (frame * 37 + 64) & 255
    m = region == 0
    r[m] = flat
    g[m] = flat
    b[m] = flat
    # region 1: gradient + noise
    m = region == 1
    r[m] = np.broadcast_to(gx, shape)[m] + n[m]
    g[m] = np.broadcast_to(gy, shape)[m] + n[m]
    b[m] = ((np.broadcast_to(xi, shape) ^ np.broadcast_to(yi, shape)) & 255)[m]
    # region 2: white noise
    m = region == 2
    r[m] = ((h >> np.uint64(8)) & np.uint64(255)).astype(np.int64)[m]
    g[m] = ((h >> np.uint64(16)) & np.uint64(255)).astype(np.int64)[m]
    b[m] = ((h >> np.uint64(24)) & np.uint64(255)).astype(np.int64)[m]
    # region 3: 45-degree stripes
    m = region == 3
    v = np.where((((xi + yi + frame) >> 2) & 1) != 0, 235, 20)
    v = np.broadcast_to(v, shape)[m]
    r[m] = v
    g[m] = v
    b[m] = v
    out = np.empty((height, width, 4), np.uint8)
    out[..., 0] = np.clip(r, 0, 255)
    out[..., 1] = np.clip(g, 0, 255)
    out[..., 2] = np.clip(b, 0, 255)
    out[..., 3] = 255
    return out
