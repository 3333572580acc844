"""libwebp_amd: MI355X-native batched WebP lossy encoder.

The product is the C-ABI shared library libwebp_amd/libwebp_amd.so
(include/webp/encode.h = the libwebp encoder ABI, include/webp/encode_gpu.h =
the batched extension). This module is a thin ctypes host binding that mirrors
the reference's calling convention: WebPConfig / WebPPicture / WebPEncode for
single pictures, and GpuBatch for HBM-resident frame batches. There is no CPU
fallback: if the shared library or the GPU is missing, calls raise.
"""
import ctypes as C
import os

from . import abi

__all__ = ["load", "GpuBatch", "encode_rgba", "device_count", "host_cpus", "lib_path", "abi"]

_HERE = os.path.dirname(os.path.abspath(__file__))
_lib = None


def lib_path():
    # WEBP_AMD_LIB selects a diagnostic build (e.g. the K3 sub-stage profile)
    return os.environ.get("WEBP_AMD_LIB") or os.path.join(_HERE, "libwebp_amd.so")


def load():
    """Load and bind libwebp_amd.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    path = lib_path()
    if not os.path.exists(path):
        raise RuntimeError("libwebp_amd.so is not built: run __graft_entry__.build() "
                           "(make -C libwebp_amd/csrc)")
    # One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64
    # (same soname as /opt/rocm's). Loading torch's first makes this
    # library bind to it, so HBM tensors, streams and our kernels share one
    # runtime; a C caller without torch simply gets /opt/rocm's.
    try:
        import torch  # noqa: F401
        if torch.version.hip is not None:
            torch.cuda.is_available()
    except ImportError:
        pass
    lib = C.CDLL(path)
    abi.bind_encoder_api(lib)
    vp, i, sz = C.c_void_p, C.c_int, C.c_size_t
    sig = {
        "WebPGpuBatchNew": (vp, [i, i, i, i, C.POINTER(abi.WebPConfig), i]),
        "WebPGpuBatchDelete": (None, [vp]),
        "WebPGpuBatchEncodeRGBA": (i, [vp, vp, sz, i, i, vp]),
        "WebPGpuBatchEncodeRGBAHost": (i, [vp, vp, sz, i, i]),
        "WebPGpuBatchEncodeRGBAHostPrefetch": (i, [vp, vp, vp, sz, i, i]),
        "WebPGpuBatchOutputSize": (sz, [vp, i]),
        "WebPGpuBatchOutput": (vp, [vp, i]),
        "WebPGpuBatchError": (i, [vp, i]),
        "WebPGpuBatchTokenCount": (sz, [vp, i]),
        "WebPGpuBatchStageCycles": (i, [vp, i, C.POINTER(C.c_uint64)]),
        "WebPGpuBatchTimings": (None, [vp, C.POINTER(C.c_double)]),
        "WebPGpuBatchGetYUV": (i, [vp, i, vp]),
        "WebPGpuBatchGetMBInfo": (i, [vp, i, vp]),
        "WebPGpuBatchGetTokens": (i, [vp, i, vp, sz]),
        "WebPGpuSynthRGBA": (i, [vp, sz, i, i, i, i, i, vp]),
        "WebPGpuDeviceCount": (i, []),
        "WebPGpuHostCpus": (i, [i, C.POINTER(C.c_int), i]),
        "WebPGpuHostThreadBudget": (i, [i, C.POINTER(C.c_int)]),
        "WebPGpuLastError": (C.c_char_p, []),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def last_error():
    return load().WebPGpuLastError().decode()


def device_count():
    return load().WebPGpuDeviceCount()


def encode_rgba(rgba, quality=75.0, method=4, stats=False, **kw):
    """Single-picture encode through the libwebp ABI (WebPPictureImportRGBA +
    WebPEncode) of libwebp_amd.so. Returns bytes (and WebPAuxStats)."""
    data, st = abi.encode_rgba(load(), rgba, quality=quality, method=method, stats=True, **kw)
    return (data, st) if stats else data


class GpuBatch:
    """Batched encoder for same-sized frames (include/webp/encode_gpu.h)."""

    def __init__(self, width, height, max_frames, quality=75.0, method=4, device=0,
                 threads=0, **cfg):
        lib = load()
        self._lib = lib
        self.width, self.height, self.max_frames = width, height, max_frames
        self.config = abi.make_config(lib, quality, method, **cfg)
        h = lib.WebPGpuBatchNew(device, width, height, max_frames, C.byref(self.config), threads)
        if not h:
            raise RuntimeError("WebPGpuBatchNew failed (no GPU, bad config or out of memory)")
        self._h = h
        self.n = 0

    def close(self):
        if getattr(self, "_h", None):
            self._lib.WebPGpuBatchDelete(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def encode_device(self, rgba_ptr, n, frame_stride=None, row_stride=None, stream=None):
        """Encode n RGBA frames at device address rgba_ptr (HBM resident)."""
        row_stride = row_stride or 4 * self.width
        frame_stride = frame_stride or row_stride * self.height
        ok = self._lib.WebPGpuBatchEncodeRGBA(self._h, rgba_ptr, frame_stride, row_stride, n,
                                              stream)
        if not ok:
            raise RuntimeError("WebPGpuBatchEncodeRGBA failed: %s" % last_error())
        self.n = n
        return self

    def encode_host_ptr(self, ptr, n, frame_stride=None, row_stride=None, next_ptr=None):
        """Encode n RGBA frames at host address ptr. Page-locked memory
        (hipHostMalloc, torch pin_memory) is uploaded by one copy on an SDMA
        engine (host/h2d_sdma.c) ahead of the encoder's kernels; pageable
        memory is copied synchronously first. next_ptr (page-locked, same
        geometry): the next batch, uploaded while this one encodes
        (WebPGpuBatchEncodeRGBAHostPrefetch); the next call with ptr ==
        next_ptr encodes from that copy."""
        row_stride = row_stride or 4 * self.width
        frame_stride = frame_stride or row_stride * self.height
        if next_ptr is not None:
            ok = self._lib.WebPGpuBatchEncodeRGBAHostPrefetch(self._h, ptr, next_ptr, frame_stride,
                                                             row_stride, n)
        else:
            ok = self._lib.WebPGpuBatchEncodeRGBAHost(self._h, ptr, frame_stride, row_stride, n)
        if not ok:
            raise RuntimeError("WebPGpuBatchEncodeRGBAHost failed: %s" % last_error())
        self.n = n

    def encode_host(self, frames):
        """frames: (N, H, W, 4) uint8 numpy array in host memory."""
        import numpy as np
        frames = np.ascontiguousarray(frames, dtype=np.uint8)
        n, h, w = frames.shape[:3]
        fs = h * w * 4          # a size-1 leading axis may carry stride 0
        assert frames.strides[1:] == (4 * w, 4, 1)
        ok = self._lib.WebPGpuBatchEncodeRGBAHost(self._h, frames.ctypes.data, fs, 4 * w, n)
        if not ok:
            raise RuntimeError("WebPGpuBatchEncodeRGBAHost failed: %s" % last_error())
        self.n = n
        return self

    def error(self, f):
        return self._lib.WebPGpuBatchError(self._h, f)

    def output(self, f):
        err = self.error(f)
        if err:
            raise RuntimeError("frame %d: %s" % (f, abi.ENC_ERRORS[err]))
        size = self._lib.WebPGpuBatchOutputSize(self._h, f)
        return C.string_at(self._lib.WebPGpuBatchOutput(self._h, f), size)

    def stage_cycles(self, f):
        c = (C.c_uint64 * 8)()
        self._lib.WebPGpuBatchStageCycles(self._h, f, c)
        return list(c)

    def token_count(self, f):
        return self._lib.WebPGpuBatchTokenCount(self._h, f)

    def output_size(self, f):
        return self._lib.WebPGpuBatchOutputSize(self._h, f)

    def outputs(self):
        return [self.output(f) for f in range(self.n)]

    def timings(self):
        t = (C.c_double * 10)()
        self._lib.WebPGpuBatchTimings(self._h, t)
        return list(t)

    def yuv(self, f):
        import numpy as np
        w, h = self.width, self.height
        uw, uh = (w + 1) // 2, (h + 1) // 2
        buf = np.empty(w * h + 2 * uw * uh, np.uint8)
        if not self._lib.WebPGpuBatchGetYUV(self._h, f, buf.ctypes.data):
            raise RuntimeError("GetYUV failed")
        y = buf[:w * h].reshape(h, w)
        u = buf[w * h:w * h + uw * uh].reshape(uh, uw)
        v = buf[w * h + uw * uh:].reshape(uh, uw)
        return y, u, v

    def mbinfo(self, f):
        import numpy as np
        nmb = ((self.width + 15) // 16) * ((self.height + 15) // 16)
        buf = np.empty((nmb, 20), np.uint8)
        if not self._lib.WebPGpuBatchGetMBInfo(self._h, f, buf.ctypes.data):
            raise RuntimeError("GetMBInfo failed")
        return buf


def host_cpus(device):
    """CPU ids the engines on `device` pin their host threads to ([] = unpinned)."""
    lib = load()
    n = lib.WebPGpuHostCpus(device, None, 0)
    buf = (C.c_int * max(n, 1))()
    n = lib.WebPGpuHostCpus(device, buf, n)
    return list(buf[:n])


def host_thread_budget(device):
    """(budget, busy): the rank's host-thread pool size on `device` (cgroup
    quota over LOCAL_WORLD_SIZE, pinned CPUs) and the threads in host phases."""
    busy = C.c_int(0)
    n = load().WebPGpuHostThreadBudget(device, C.byref(busy))
    return n, busy.value


def synth_device(ptr, width, height, first, n, seed=1, frame_stride=None, stream=None):
    """Fill device memory with syn-v1 frames (benchmark input generator)."""
    fs = frame_stride or 4 * width * height
    if not load().WebPGpuSynthRGBA(ptr, fs, width, height, first, n, seed, stream):
        raise RuntimeError("WebPGpuSynthRGBA failed")
