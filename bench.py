#!/usr/bin/env python3
"""Benchmark: batched WebP lossy encode (cwebp -q 75 -m 4) of 1920x1080 RGBA
frames on MI355X, BASELINE.json configs[1] (1 GPU) / configs[2] (8 GPUs).

One "step" = one batch of the rank's syn-v1 frames taken from
RGBA in pinned host memory to .webp byte strings in host memory: the H2D
upload, K1 import, K2 analysis, host segment setup, K3 RD search + tokens, K4
boolean coder on the device (host codes partition 0 meanwhile), one D2H of
the packed partitions and the RIFF write. `value` is that rate, SURVEY.md
8(d)'s own MP/s definition (upload included): each encoder instance uploads
its step i+1 on a copy stream while its step i encodes. The same frames
already resident in HBM (no upload) are timed after it as `hbm_resident_mps`.

Multi-GPU (configs[2]): one process per GPU. `--gpus N` without a torchrun
environment starts `torch.distributed.run` with N ranks itself (a child
process, before this process touches the GPU) and exits with its status.
Rank r encodes frames [r*B, (r+1)*B); the only data-path collective is an
all-gather of the encoded sizes (RCCL), plus the barrier / max-over-ranks
timing of the harness contract. After the timed loop every rank checks the
frames of its timed batch that tests/golden/shard_kat.json pins (reference
libwebp SHA-256s) and rank 0 reports the result as `kat_check`.

`--stub` replaces the GPU encoder by a CPU test double (gloo backend): the
launcher, sharding, size gather and timing run exactly as on the GPU
(tests/test_bench_dist.py).
"""
import argparse
import hashlib
import json
import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E peak (MI355X_MICROARCH.md)
BOX_CORE_SHARE = 16     # host cores the GPU pool grants a one-GPU job (its operator notes)


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks; without a torchrun environment bench.py launches them itself")
    ap.add_argument("--steps", type=int, default=0,
                    help="timed steps (0: three per encoder instance, 12 lossy / 9 lossless, so "
                         "the line is not dominated by filling and draining the pipeline)")
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=0,
                    help="frames per GPU per step (0: 256 lossy, 1024 lossless)")
    ap.add_argument("--lossless", action="store_true",
                    help="configs[4]: -lossless -m 4 (VP8L) instead of the lossy headline")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--quality", type=float, default=75.0)
    ap.add_argument("--method", type=int, default=4)
    ap.add_argument("--sharp-yuv", action="store_true",
                    help="use_sharp_yuv import (cwebp -sharp_yuv); not the headline config")
    ap.add_argument("--low-memory", action="store_true",
                    help="config->low_memory (cwebp -low_memory, VP8EncLoop); not the headline")
    ap.add_argument("--threads", type=int, default=0, help="host tail threads (0 = auto)")
    ap.add_argument("--engines", type=int, default=0,
                    help="encoder instances on their own streams and host threads; steps are "
                         "dealt round-robin so one batch's host work overlaps another's kernels "
                         "(0: 6 lossy -- with the double-buffered upload 4321-4435 MP/s with 4, "
                         "4446-4465 with 5, 4494-4497 with 6, profiles/r4/pf2; 8 gave 4535-4546 "
                         "against 4409-4533 for 6 on one box, profiles/r4/eng68: kept at 6 for "
                         "the host threads of 8 ranks on one node; 3 lossless -- "
                         "profiles/r3/lab_*.json)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="CPU work per baseline leg (single thread, all cores)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--input", choices=("host", "hbm"), default="host",
                    help="timed steps take RGBA from pinned host memory (upload included, "
                         "SURVEY.md 8(d), the default) or already resident in HBM")
    ap.add_argument("--no-host-input", dest="input", action="store_const", const="hbm",
                    help="same as --input hbm")
    ap.add_argument("--no-prefetch", dest="prefetch", action="store_false",
                    help="host input: upload each batch inside its own call only (no "
                         "upload of an engine's next batch while its current one encodes)")
    ap.add_argument("--no-other-input", action="store_true",
                    help="skip timing the other input mode after the line's steps")
    ap.add_argument("--stub", action="store_true",
                    help="CPU test double instead of the GPU encoder (gloo; tests only)")
    ap.add_argument("--dist-backend", choices=("nccl", "gloo"), default=None,
                    help="collective backend (default nccl = RCCL on the GPUs; gloo lets "
                         "tests run several real-encoder ranks on one GPU)")
    ap.add_argument("--same-device", action="store_true",
                    help="every rank on device 0 (tests on a one-GPU box only)")
    ap.add_argument("--force-pg", action="store_true",
                    help="create the process group (and run the size all-gather / timing "
                         "reductions through it) even with one rank (tests of the RCCL path)")
    return ap.parse_args(argv)


# ---------------------------------------------------------------------------
# launcher

def launch_ranks(args, argv):
    """--gpus N > 1 outside torchrun: run N ranks through torch.distributed.run
    as a child process and return its exit status (None: run in-process)."""
    if args.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return None
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node", str(args.gpus), "--master-addr", "127.0.0.1",
           "--master-port", str(port), os.path.abspath(__file__)] + list(argv)
    return subprocess.call(cmd)


# ---------------------------------------------------------------------------
# CPU baseline: the reference libwebp (oracle/_ref, built from /root/reference
# sources by oracle/Makefile) on this host's cores

def _ref_encoder(quality, method, lossless):
    import ctypes as C
    from libwebp_amd import abi
    ref = os.path.join(HERE, "oracle", "_ref", "libwebp_ref.so")
    if os.path.exists(ref):
        lib = abi.bind_encoder_api(C.CDLL(ref))
        kw = {"lossless": 1, "use_argb": True} if lossless else {}
        return "reference", lambda img: abi.encode_rgba(lib, img, quality=quality,
                                                        method=method, **kw)
    if lossless:
        return None, None
    from oracle import oracle as orc   # the C restatement, also single-threaded
    return "port", lambda img: orc.encode_rgba(img, quality=quality, method=method)


def _cpu_leg(width, height, quality, method, lossless, seconds, first):
    """Encode syn-v1 frames first, first+1, ... for `seconds` of wall time
    (after one untimed warm-up frame); returns (frames, seconds, kind)."""
    from libwebp_amd.synth import syn_v1
    kind, enc = _ref_encoder(quality, method, lossless)
    if enc is None:
        return 0, 0.0, None
    imgs = [syn_v1(width, height, first + k) for k in range(2)]
    enc(imgs[0])
    frames, t0 = 0, time.perf_counter()
    while True:
        enc(imgs[frames & 1])
        frames += 1
        el = time.perf_counter() - t0
        if el >= seconds and frames >= 2:
            return frames, el, kind


def _cpu_leg_worker(a):
    return _cpu_leg(*a)


def cgroup_cpu_quota():
    """CPUs granted by the cgroup CPU quota (v2 cpu.max, v1 cfs_quota), or None."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            return int(q) / int(per)
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        if q > 0:
            return q / per
    except (OSError, ValueError):
        pass
    return None


def cpu_share():
    """(processes for the all-cores CPU leg, why that many): the cgroup CPU
    quota when one is set, else the process's affinity set, in both cases at
    most the pool's per-GPU core share (BOX_CORE_SHARE)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    quota = cgroup_cpu_quota()
    if quota is not None:
        n = max(1, min(aff, int(quota + 0.5)))
        why = "cgroup CPU quota %.1f CPUs, affinity set %d CPUs" % (quota, aff)
    else:
        n = aff
        why = "no cgroup CPU quota, affinity set %d CPUs" % aff
    if n > BOX_CORE_SHARE:
        why += "; capped at the pool's per-GPU share of %d cores" % BOX_CORE_SHARE
        n = BOX_CORE_SHARE
    return n, why


def cpu_baseline(width, height, quality, method, seconds, lossless=False):
    """WebPPictureImportRGBA + WebPEncode into a memory writer,
    single thread (the 40x denominator) and one process per host core
    (independent frames). Runs before this process touches the GPU (the
    all-core leg forks)."""
    import multiprocessing as mp
    frames, el, kind = _cpu_leg(width, height, quality, method, lossless, seconds, 1)
    if kind is None:
        return None
    px = width * height
    cores, share_note = cpu_share()
    with mp.get_context("fork").Pool(cores) as pool:
        legs = pool.map(_cpu_leg_worker, [(width, height, quality, method, lossless, seconds,
                                           1 + 2 * k) for k in range(cores)])
    all_frames = sum(l[0] for l in legs)
    all_wall = max(l[1] for l in legs)
    mode = " lossless" if lossless else ""
    return {"value": round(frames * px / el / 1e6, 3), "unit": "MP/s", "cores": 1,
            "kind": kind,
            "sample": "%d syn-v1 %dx%d frames, q%d m%d%s, WebPPictureImportRGBA+WebPEncode, "
                      "single thread, %.1f s" % (frames, width, height, quality, method, mode, el),
            "all_cores": {"value": round(all_frames * px / all_wall / 1e6, 3), "unit": "MP/s",
                          "cores": cores, "cores_basis": share_note,
                          "sample": "%d processes x %.1f s, %d frames in all, independent "
                                    "frames per process" % (cores, all_wall, all_frames)}}


# ---------------------------------------------------------------------------
# multi-rank plumbing (any backend: nccl on the GPUs, gloo in the CPU tests)

def shard(rank, frames_per_rank):
    """Frames [first, first + n) owned by `rank`."""
    return rank * frames_per_rank, frames_per_rank


def gather_sizes(sizes, world):
    """All-gather the per-frame encoded sizes of every rank (the only
    data-path collective)."""
    import torch
    import torch.distributed as dist
    if not dist.is_initialized():
        return [sizes]
    out = [torch.empty_like(sizes) for _ in range(world)]
    dist.all_gather(out, sizes)
    return out


def max_over_ranks(seconds, world, device):
    import torch
    import torch.distributed as dist
    if not dist.is_initialized():
        return seconds
    t = torch.tensor([seconds], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(values, world, device):
    import torch
    import torch.distributed as dist
    t = torch.tensor(values, dtype=torch.int64, device=device)
    if dist.is_initialized():
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return [int(v) for v in t.tolist()]


def shard_kats(args):
    """Known answers (frame -> sha256) for the default lossy workload, or {}."""
    path = os.path.join(HERE, "tests", "golden", "shard_kat.json")
    if (args.lossless or args.sharp_yuv or args.low_memory or not os.path.exists(path)):
        return {}
    k = json.load(open(path))
    if (k["width"], k["height"], k["quality"], k["method"]) != (
            args.width, args.height, args.quality, args.method):
        return {}
    if args.stub:   # the same frames, with the test double's own answers
        return {int(f): hashlib.sha256(StubBatch(0).output(int(f))).hexdigest()
                for f in k["frames"]}
    return {int(f): v["sha256"] for f, v in k["frames"].items()}


class StubBatch:
    """CPU test double with GpuBatch's interface (tests only): 'encodes' frame
    f into a deterministic 100 + f % 7 byte string, taking ~1 ms per step."""

    def __init__(self, first):
        self.first, self.n = first, 0

    def encode_device(self, ptr, n, stream=None):
        time.sleep(0.001)
        self.n = n

    def output(self, f):
        g = self.first + f
        return bytes([g & 255]) * (100 + g % 7)

    def output_size(self, f):
        return len(self.output(f))

    def error(self, f):
        return 0

    def token_count(self, f):
        return 0

    def timings(self):
        return [0.0] * 10

    def close(self):
        pass


# ---------------------------------------------------------------------------

def lossless_line(args, world, B, W, H, elapsed, tails, total_bytes, solo=None):
    """configs[4] line: VP8L encode. Dominant kernel: the L1 transform tile
    kernel (k_vp8l_transform_w: one wave per 8..32-pixel tile, or
    k_vp8l_transform for 4- and 64-pixel tiles); algorithmic bytes per launch
    = RGBA read (4 B/px) + residual ARGB written (4 B/px) + per-tile
    modes/multipliers."""
    mp_ = world * B * W * H * args.steps / 1e6
    steps = len(tails)
    avg = lambda i: sum(t[i] for t in tails) / steps
    tb = 5 if args.method == 4 else (6 if args.method < 4 else 4)
    ntt = ((W + (1 << tb) - 1) >> tb) * ((H + (1 << tb) - 1) >> tb)
    l1_bytes = B * (8 * W * H + 5 * ntt)
    l1_s = avg(7) / 1e6
    l1_solo = solo[7] / 1e6 if solo else l1_s
    achieved = l1_bytes / l1_solo / 1e9 if l1_solo > 0 else 0.0
    # PMC bytes of one k_vp8l_transform launch of this workload (a step is one
    # instance's call on the whole batch)
    l1_kernel = "k_vp8l_transform_w" if 3 <= tb <= 5 else "k_vp8l_transform"
    l1_traffic, l1_tsrc = measured_traffic(l1_kernel, B, W, H, args.quality,
                                           args.method, lossless=True)
    return {
        "metric": "megapixels/sec encoded (cwebp -lossless -m 4, 1920x1080 batch)",
        "value": round(mp_ / elapsed, 3),
        "unit": "MP/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8/u32",
        "data": "synthetic syn-v1 RGBA frames (SURVEY.md 8(d)), generated on the device",
        "config": {"workload": "batch of %d %dx%d RGBA frames per GPU, -lossless -q %g -m %d" %
                               (B, W, H, args.quality, args.method),
                   "frames_per_gpu": B, "width": W, "height": H, "quality": args.quality,
                   "method": args.method, "parallelism": "frames sharded %d ways" % world,
                   "engines_per_gpu": getattr(args, "engines_used", 1)},
        "roofline": {"bound": "hbm", "kernel": l1_kernel, "achieved": round(achieved, 3),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": l1_traffic,
                     "traffic_source": l1_tsrc,
                     "k_ms": round(1e3 * l1_s, 3), "k_solo_ms": round(1e3 * l1_solo, 3),
                     "algorithmic_bytes_per_launch": l1_bytes,
                     # the per-frame-serial kernels (one wave / one workgroup per
                     # frame): their share is k_cache_parse_cluster_events below
                     "per_frame_serial_kernels": ["k_vp8l_cache (one wave per frame segment, "
                                                  "up to 16 segments)",
                                                  "k_vp8l_cluster (one workgroup per frame)",
                                                  "k_vp8l_predsel (one workgroup per frame, "
                                                  "near-lossless / transparent frames only)"]},
        "stage_ms": {k: round(avg(i) / 1e3, 3) for k, i in
                     (("transform_analysis", 0), ("host_headers", 1), ("bit_writer", 2),
                      ("d2h", 3), ("riff", 4), ("total", 5), ("k_transform_events", 7),
                      ("k_cache_parse_cluster_events", 6), ("k_write_events", 8))},
        "output_bytes_per_frame": round(total_bytes / (world * B), 1),
    }


def issue_roofline(B, W, H, quality, method, k3_seconds):
    """K3's vector-issue fraction: SQ_INSTS_VALU per launch and the effective
    clock from the committed SQ passes of this same workload
    (profiles/k3_issue.json, tools/k3_issue.py) over 1024 SIMDs x 0.5 wave64
    VALU instructions per cycle x this run's solo K3 time; None for another
    workload."""
    path = os.path.join(HERE, "profiles", "k3_issue.json")
    if not os.path.exists(path) or (B, W, H, quality, method) != (256, 1920, 1080, 75.0, 4) \
            or k3_seconds <= 0:
        return None
    d = json.load(open(path))
    peak = 1024 * 0.5 * d["effective_clock_hz"]
    return {"achieved": round(d["valu_per_launch"] / k3_seconds / 1e12, 4),
            "peak": round(peak / 1e12, 4), "unit": "T wave64 VALU instructions/s",
            "frac": round(d["valu_per_launch"] / (peak * k3_seconds), 4),
            "frac_profiled": round(d["issue_frac_profiled"], 4),
            "lane_utilisation": round(d["lane_utilisation"], 4),
            "valu_per_launch": d["valu_per_launch"],
            "effective_clock_hz": round(d["effective_clock_hz"]), "source": d["source"]}


def measured_traffic(kernel, B, W, H, quality, method, lossless=False):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC passes
    (profiles/hbm_traffic.json, profiles/hbm_traffic_lossless.json: FETCH_SIZE
    and WRITE_SIZE of one launch of this same default workload, gfx950
    corrections applied as documented there), or None for another workload."""
    path = os.path.join(HERE, "profiles",
                        "hbm_traffic_lossless.json" if lossless else "hbm_traffic.json")
    want = (1024 if lossless else 256, 1920, 1080, 75.0, 4)
    if not os.path.exists(path) or (B, W, H, quality, method) != want:
        return None, None
    d = json.load(open(path))
    k = d["kernels"].get(kernel)
    return (int(k["bytes_per_launch"]) if k else None), d["source"]


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse_args(argv)
    rc = launch_ranks(args, argv)
    if rc is not None:
        return rc

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if "WORLD_SIZE" in os.environ and args.gpus not in (1, world):
        raise SystemExit("--gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    W, H = args.width, args.height
    B = args.batch or (1024 if args.lossless else 256)
    if not args.engines:
        # lossy: 6 instances with the double-buffered upload (4494-4497 MP/s
        # against 4446-4465 with 5 and 4321-4435 with 4, profiles/r4/pf2)
        args.engines = 3 if args.lossless else 6
    if not args.steps:
        args.steps = 3 * (1 if args.stub else args.engines)

    # the CPU baseline first: before this process initialises the GPU
    cb = None
    if rank == 0 and world == 1 and not args.no_cpu and not args.stub:
        cb = cpu_baseline(W, H, int(args.quality), args.method, args.cpu_seconds,
                          lossless=args.lossless)

    import torch
    import torch.distributed as dist
    gpu_dev = 0 if args.same_device else local
    if args.stub:
        dev = torch.device("cpu")
        backend = "gloo"
    else:
        torch.cuda.set_device(gpu_dev)
        dev = torch.device("cuda", gpu_dev)
        backend = args.dist_backend or "nccl"
    # the collectives' tensors: on the GPU for RCCL, in host memory for gloo
    cdev = dev if backend == "nccl" else torch.device("cpu")
    if world > 1 or args.force_pg:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if "MASTER_PORT" not in os.environ:   # a one-rank group outside torchrun
            import socket
            sk = socket.socket()
            sk.bind(("127.0.0.1", 0))
            os.environ["MASTER_PORT"] = str(sk.getsockname()[1])
            sk.close()
        if backend == "nccl":
            dist.init_process_group(backend, rank=rank, world_size=world, device_id=dev)
        else:
            dist.init_process_group(backend, rank=rank, world_size=world)
    cpus = []
    if not args.stub:
        # this rank's host threads on its GPU's NUMA node; the
        # engines pin their own worker threads to the same CPUs
        import libwebp_amd
        cpus = libwebp_amd.host_cpus(gpu_dev)
        if cpus:
            os.sched_setaffinity(0, cpus)

    first, _ = shard(rank, B)
    if args.stub:
        rgba, stream, enc = None, None, StubBatch(first)
    else:
        import libwebp_amd
        rgba = torch.empty(B * 4 * W * H, dtype=torch.uint8, device=dev)
        stream = torch.cuda.current_stream(dev).cuda_stream
        libwebp_amd.synth_device(rgba.data_ptr(), W, H, first, B, seed=1, stream=stream)
        torch.cuda.synchronize(dev)
        enc = libwebp_amd.GpuBatch(W, H, B, quality=args.quality, method=args.method,
                                   device=gpu_dev, threads=args.threads,
                                   use_sharp_yuv=int(args.sharp_yuv),
                                   lossless=int(args.lossless), low_memory=int(args.low_memory))

    # more engines: each on its own HIP stream with its own host buffers; the
    # timed steps are dealt round-robin to one host thread per engine (the
    # ctypes calls release the GIL), so one batch's host stages (segment
    # setup, partition 0, RIFF write) run while another batch's kernels do
    E = 1 if args.stub else max(1, min(args.engines, args.steps))
    args.engines_used = E
    encs = [enc]
    for _ in range(E - 1):
        encs.append(libwebp_amd.GpuBatch(W, H, B, quality=args.quality, method=args.method,
                                         device=gpu_dev, threads=args.threads,
                                         use_sharp_yuv=int(args.sharp_yuv),
                                         lossless=int(args.lossless),
                                         low_memory=int(args.low_memory)))

    # input of a step: "host" = RGBA in pinned host memory, uploaded by the
    # step itself: WebPGpuBatchEncodeRGBAHostPrefetch copies
    # the batch with a blocking HSA SDMA transfer under a per-device mutex
    # (host/h2d_sdma.c: a copy engine, no CU) unless the previous call already
    # prefetched it, and starts the next batch's SDMA copy into the engine's
    # spare buffer, which then overlaps the current batch's kernels and host
    # stages; "hbm" = the frames already in HBM
    host_in = args.input == "host" and not args.stub
    pinned = None

    def make_pinned():
        p = torch.empty(rgba.numel(), dtype=torch.uint8, pin_memory=True)
        p.copy_(rgba)
        return p

    if host_in:
        pinned = make_pinned()

    def engine_steps(e, n, host, tails):
        """Engine e's share of n steps (dealt round-robin over the engines)."""
        mine = range(e, n, E)
        for k, _ in enumerate(mine):
            if host:
                # double-buffered upload: while this batch encodes, the engine's
                # next batch of the same run goes up on a copy engine. Every
                # batch of the timed run is uploaded inside it: its first call
                # uploads its own frames and its last starts no upload.
                nxt = pinned.data_ptr() if args.prefetch and k + 1 < len(mine) else None
                encs[e].encode_host_ptr(pinned.data_ptr(), B, next_ptr=nxt)
            else:
                encs[e].encode_device(rgba.data_ptr() if rgba is not None else 0, B,
                                      stream=stream)
            if tails is not None:
                tails.append(encs[e].timings())

    def barrier():
        if dist.is_initialized():
            dist.barrier()
        if not args.stub:
            torch.cuda.synchronize(dev)

    def run(n, host, tails=None):
        """n steps over the E engines (one host thread each when E > 1; the
        ctypes calls release the GIL), bracketed by barrier + synchronize;
        returns the wall time."""
        barrier()
        t0 = time.perf_counter()
        if E == 1:
            engine_steps(0, n, host, tails)
        else:
            import threading
            errors = []

            def worker(e):
                try:
                    engine_steps(e, n, host, tails)
                except Exception as ex:   # re-raised below, after every thread ends
                    errors.append(ex)

            th = [threading.Thread(target=worker, args=(e,)) for e in range(E)]
            for t in th:
                t.start()
            for t in th:
                t.join()
            if errors:
                raise errors[0]
        barrier()
        return time.perf_counter() - t0

    run(E * max(args.warmup, 1 if E > 1 else 0), host_in)
    tails = []
    elapsed = run(args.steps, host_in, tails)

    errs = [enc.error(f) for f in range(B)]
    if any(errs):
        raise RuntimeError("rank %d: frame errors %s" % (rank, sorted(set(errs))))
    # parity of the timed batch: the frames the reference's known answers pin
    kats = shard_kats(args)
    checked = failed = 0
    for g, want in kats.items():
        if first <= g < first + B:
            checked += 1
            failed += hashlib.sha256(enc.output(g - first)).hexdigest() != want
    sizes = torch.tensor([enc.output_size(f) for f in range(B)], dtype=torch.int64, device=cdev)
    ntok = sum(enc.token_count(f) for f in range(B))
    allsizes = gather_sizes(sizes, world)
    elapsed = max_over_ranks(elapsed, world, cdev)
    checked, failed = sum_over_ranks([checked, failed], world, cdev)
    total_bytes = int(sum(int(s.sum().item()) for s in allsizes))

    # the dominant kernel's time without the other instances' kernels beside
    # it: one more (untimed) HBM-input step on instance 0 alone -- with several
    # instances the HIP events of the timed steps include waiting for CUs the
    # other instances' kernels hold
    solo = None
    if not args.stub:
        barrier()
        engine_steps(0, 1, False, None)
        barrier()
        solo = enc.timings()
    # the other input mode, reported beside the line (HBM-resident input when
    # the timed steps uploaded from host memory, and vice versa)
    other_rate = None
    if not args.stub and not args.no_other_input:
        n_other = max(3 * E, min(args.steps, 4))
        if not host_in:
            pinned = make_pinned()
        el = max_over_ranks(run(n_other, not host_in), world, cdev)
        other_rate = world * n_other * B * W * H / el / 1e6
    del pinned

    # device memory in use with every instance's buffers allocated and run
    # (the whole device: a box runs one job)
    hbm_used = None
    if not args.stub:
        free_b, total_b = torch.cuda.mem_get_info(dev)
        hbm_used = round((total_b - free_b) / 1e9, 2)
    line = None
    if rank == 0:
        if args.lossless:
            line = lossless_line(args, world, B, W, H, elapsed, tails, total_bytes, solo)
        else:
            line = lossy_line(args, world, B, W, H, elapsed, tails, total_bytes, ntok, solo)
        if kats and failed:
            line["kat_check"] = "FAIL: %d of %d timed-batch frames differ from " \
                                "tests/golden/shard_kat.json" % (failed, checked)
        elif kats:
            line["kat_check"] = "ok: %d timed-batch frames on %d rank(s) equal " \
                                "tests/golden/shard_kat.json" % (checked, world)
        line["config"]["input"] = "host" if host_in else "hbm"
        line["input"] = ("host: RGBA in pinned host memory -> .webp in host memory, H2D "
                         "upload of every step inside the timed run (SURVEY.md 8(d)): one "
                         "copy on an SDMA engine, beside the other %d instance(s)' kernels; "
                         "%s" % (len(encs) - 1,
                                 "double-buffered: an instance's next batch goes up while its "
                                 "current one encodes (the run's first batch per instance "
                                 "uploads in its own call, its last starts no upload)"
                                 if args.prefetch else "each batch uploaded in its own call")
                         if host_in else
                         "hbm: RGBA frames already resident in HBM (no upload)")
        if other_rate is not None:
            key = "hbm_resident_mps" if host_in else "host_input_mps"
            line[key] = round(other_rate, 3)
        if cb:
            line["cpu_baseline"] = cb
        if not args.stub:
            line["host_cpus_per_rank"] = len(cpus) if cpus else "unpinned"
            line["host_threads_per_rank"] = {
                "budget": libwebp_amd.host_thread_budget(gpu_dev)[0],
                "engines": len(encs),
                "note": "every engine of the rank draws its host-phase helper threads from "
                        "one pool of `budget` threads (cgroup quota / LOCAL_WORLD_SIZE, "
                        "pinned CPUs; host/host_cpus.c)"}
            if hbm_used is not None:
                line["hbm_used_gb"] = hbm_used
        if args.stub:
            line["data"] = "stub encoder (CPU test double, no GPU)"
        if dist.is_initialized():
            line["collectives"] = "%s, %d rank(s): all-gather of the encoded sizes, " \
                                  "max / sum reductions" % (dist.get_backend(), world)
        print(json.dumps(line), flush=True)
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()
    for e in encs:
        e.close()
    if failed:
        raise SystemExit("timed-batch frames differ from the reference known answers")
    return 0


def lossy_line(args, world, B, W, H, elapsed, tails, total_bytes, ntok, solo=None):
    mp_ = world * B * W * H * args.steps / 1e6
    steps = len(tails)
    avg = lambda i: sum(t[i] for t in tails) / steps
    # K3 (k_encode) roofline: algorithmic bytes per launch = YUV420 planes read
    # (W*H + 2*ceil(W/2)*ceil(H/2) per frame) + 16-bit token stream written +
    # 20 B/MB mode info + the per-frame result block.
    nmb = ((W + 15) // 16) * ((H + 15) // 16)
    yuv = W * H + 2 * ((W + 1) // 2) * ((H + 1) // 2)
    k3_bytes = B * (yuv + 20 * nmb + 1160) + 2 * ntok
    k3_s = avg(6) / 1e6
    k3_solo = solo[6] / 1e6 if solo else k3_s   # the roofline uses the uncontended time
    achieved = k3_bytes / k3_solo / 1e9 if k3_solo > 0 else 0.0
    # SURVEY.md 8(d)'s unit: 7 W H + coded bytes per frame (RGBA read, YUV
    # written and read back, the file), over the same K3 time
    s8d_bytes = int(B * (7 * W * H + total_bytes / (world * B)))
    s8d_achieved = s8d_bytes / k3_solo / 1e9 if k3_solo > 0 else 0.0
    traffic, tsrc = (None, None)
    issue = None
    if not (args.sharp_yuv or args.low_memory or args.stub):
        traffic, tsrc = measured_traffic("k_encode", B, W, H, args.quality, args.method)
        issue = issue_roofline(B, W, H, args.quality, args.method, k3_solo)
    return {
        "metric": "megapixels/sec encoded (cwebp -q 75, 1920x1080 batch)",
        "value": round(mp_ / elapsed, 3),
        "unit": "MP/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8/int32",
        "data": "synthetic syn-v1 RGBA frames (SURVEY.md 8(d)), generated on the device",
        "config": {"workload": "batch of %d %dx%d RGBA frames per GPU, -q %g -m %d%s" %
                               (B, W, H, args.quality, args.method,
                                (" -sharp_yuv" if args.sharp_yuv else "") +
                                (" -low_memory" if args.low_memory else "")),
                   "frames_per_gpu": B, "width": W, "height": H,
                   "quality": args.quality, "method": args.method,
                   "parallelism": "frames sharded %d ways" % world,
                   "engines_per_gpu": getattr(args, "engines_used", 1)},
        "roofline": {"bound": "hbm", "kernel": "k_encode", "achieved": round(achieved, 3),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 6),
                     "traffic": traffic, "traffic_source": tsrc,
                     "k_encode_ms": round(1e3 * k3_s, 3),
                     "k_encode_solo_ms": round(1e3 * k3_solo, 3),
                     "k_encode_ms_note": "k_encode_ms: HIP events of the timed steps (with "
                                         "the other instance's kernels beside it); "
                                         "k_encode_solo_ms: one step on one instance alone, "
                                         "the time `achieved` uses (≈ rocprof's average, "
                                         "profiles/r5/final/kernel_stats_solo_r5fg.csv: 96.74 ms)",
                     "algorithmic_bytes_per_launch": k3_bytes,
                     "s8d": {"bytes_per_launch": s8d_bytes,
                             "achieved": round(s8d_achieved, 3),
                             "frac": round(s8d_achieved / HBM_PEAK_GBS, 6),
                             "note": "SURVEY.md 8(d)'s algorithmic bytes (7 W H + coded bytes "
                                     "per frame) over k_encode_solo_ms; `achieved` / `frac` "
                                     "above count K3's own reads and writes (YUV, mode info, "
                                     "results, tokens)"},
                     # the roof that binds K3: vector issue
                     "issue": issue},
        "stage_ms": {k: round(avg(i) / 1e3, 3) for k, i in
                     (("import_analysis", 0), ("host_setup", 1), ("rd_tokens", 2),
                      ("d2h", 3), ("host_tail", 4), ("total", 5),
                      ("k_encode_events", 6), ("k_import_analyze_events", 7),
                      ("k_emit_events", 8))},
        "output_bytes_per_frame": round(total_bytes / (world * B), 1),
    }


if __name__ == "__main__":
    sys.exit(main())
