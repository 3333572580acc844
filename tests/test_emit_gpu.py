"""K4 (hip/vp8_emit.hip) alone on token streams built to stress it: random
streams, streams with long runs of 1 bits, and streams that drive the
coder's low end up to a point and across it (long runs of 1 bits in N, then
a carry through them: out of k_emit_seg's 64-bit window and into the words
it already wrote), cut
at and around the 2048-token segment size. Each stream's bytes must equal
libwebp's boolean coder on the same (bit, probability) sequence
(tests/test_emit_model.py: ref_coder, a restatement of
src/utils/bit_writer_utils.c:55-124,199-206; its window model there is the
same algorithm run on CPU)."""
import ctypes as C
import random

import numpy as np
import pytest

import libwebp_amd
from test_emit_model import _carry_forcing, _carry_heavy, ref_coder, window_coder

pytestmark = pytest.mark.gpu


def _streams():
    rng = random.Random(2027)
    out = []
    for n in [0, 1, 2, 7, 2047, 2048, 2049, 4096, 6001, 20000, 100000]:
        toks = []
        for _ in range(n):
            p = rng.randint(1, 255)
            toks.append((1 if rng.random() * 256 >= p else 0, p))
        out.append(toks)
        out.append(_carry_heavy(rng, n))
        if 0 < n <= 20000:
            out.append(_carry_forcing(rng, n))
    return out


def _run(streams):
    lib = libwebp_amd.load()
    f = lib.vp8g_emit_streams
    f.restype = C.c_int
    f.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_uint32, C.c_void_p]
    flat = np.array([(b << 15) | (1 << 14) | p for s in streams for b, p in s], np.uint16)
    ntok = np.array([len(s) for s in streams], np.uint32)
    stride = int((7 * int(ntok.max()) + 48) // 8 + 16)
    out = np.zeros((len(streams), stride), np.uint8)
    size = np.zeros(len(streams), np.uint32)
    assert f(flat.ctypes.data if flat.size else None, ntok.ctypes.data, len(streams),
             out.ctypes.data, stride, size.ctypes.data) == 1
    return [out[i, :size[i]].tobytes() for i in range(len(streams))]


def test_emit_streams_match_reference_coder():
    streams = _streams()
    got = _run(streams)
    carries = {}
    for i, toks in enumerate(streams):
        want = ref_coder(toks)
        window_coder(toks, 2048, 32, carries)
        assert got[i] == want, (i, len(toks))
    assert carries.get("carries", 0) > 0   # the streams took the carry path


def _run_rows(streams, rowlen):
    """The same streams laid out as K3's token rows (vp8g_emit_rows: rows of
    rowlen tokens, rowcap = round8(rowlen) + 8 apart) and coded in place."""
    lib = libwebp_amd.load()
    f = lib.vp8g_emit_rows
    f.restype = C.c_int
    f.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_uint32, C.c_void_p, C.c_uint32, C.c_void_p]
    flat = np.array([(b << 15) | (1 << 14) | p for s in streams for b, p in s], np.uint16)
    ntok = np.array([len(s) for s in streams], np.uint32)
    stride = int((7 * int(ntok.max()) + 48) // 8 + 16)
    out = np.zeros((len(streams), stride), np.uint8)
    size = np.zeros(len(streams), np.uint32)
    assert f(flat.ctypes.data if flat.size else None, ntok.ctypes.data, len(streams), rowlen,
             out.ctypes.data, stride, size.ctypes.data) == 1
    return [out[i, :size[i]].tobytes() for i in range(len(streams))]


@pytest.mark.parametrize("rowlen", [100, 255, 256, 1001, 2048, 2050, 5003])
def test_emit_row_streams_match_reference_coder(rowlen):
    """Row streams (the token loop's layout, tokens read where K3 wrote them):
    segments cut per row, rows shorter than the 256-token look-back (the next
    segment then starts from all 128 ranges), row ends off the 8-token grid
    (the look-back read token by token), rows longer than a segment."""
    streams = _streams()
    got = _run_rows(streams, rowlen)
    for i, toks in enumerate(streams):
        assert got[i] == ref_coder(toks), (i, len(toks), rowlen)
