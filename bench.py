#!/usr/bin/env python3
"""Benchmark: batched WebP lossy encode (cwebp -q 75 -m 4) of 1920x1080 RGBA
frames on MI355X, BASELINE.json configs[1] (1 GPU) / configs[2] (8 GPUs).

One "step" = one WebPGpuBatchEncodeRGBA call over the rank's batch of
HBM-resident syn-v1 frames: K1 import, K2 analysis, host
segment setup, K3 RD search + tokens, K4 boolean coder on the device (host
codes partition 0 meanwhile), one D2H of the packed partitions and the RIFF
write, ending with every .webp in host memory. Frames are
synthesised on the device before timing starts (value = throughput with the
input resident in HBM); the PCIe-inclusive host-input rate is measured
separately by `--host-input` and documented in DESIGN.md.

Multi-GPU: one process per GPU (torchrun). Rank r encodes frames
[r*B, (r+1)*B); the only collective is an all-gather of encoded sizes (RCCL),
plus the barrier / max-over-ranks timing required by the harness.

Output: one JSON line on rank 0 (see README contract in DESIGN.md).
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def cpu_baseline(width, height, quality, method, seconds, lossless=False):
    """Reference libwebp (compiled from /root/reference sources into
    oracle/_ref by oracle/Makefile) timed single-threaded on this host:
    WebPPictureImportRGBA + WebPEncode into a memory writer, syn-v1 frames
    1, 2, ... until `seconds` of CPU work (frame 0 is an untimed warm-up)."""
    import numpy as np
    from libwebp_amd import abi
    from libwebp_amd.synth import syn_v1
    import ctypes as C
    ref = os.path.join(HERE, "oracle", "_ref", "libwebp_ref.so")
    kind = "reference"
    if os.path.exists(ref):
        lib = C.CDLL(ref)
        abi.bind_encoder_api(lib)
        if lossless:   # ARGB picture, like cwebp -lossless
            enc = lambda img: abi.encode_rgba(lib, img, quality=quality, method=method,
                                              lossless=1, use_argb=True)
        else:
            enc = lambda img: abi.encode_rgba(lib, img, quality=quality, method=method)
    elif lossless:
        return None
    else:   # the C restatement (oracle/), also single-threaded
        from oracle import oracle as orc
        kind = "port"
        enc = lambda img: orc.encode_rgba(img, quality=quality, method=method)
    enc(syn_v1(width, height, 0))
    elapsed, frames, f = 0.0, 0, 1
    while elapsed < seconds or frames < 2:
        img = syn_v1(width, height, f)
        t0 = time.perf_counter()
        enc(img)
        elapsed += time.perf_counter() - t0
        frames += 1
        f += 1
    mps = frames * width * height / elapsed / 1e6
    return {"value": round(mps, 3), "unit": "MP/s", "cores": 1, "kind": kind,
            "sample": "%d syn-v1 %dx%d frames (f=1..%d), q%d m%d%s, WebPPictureImportRGBA+"
                      "WebPEncode, single thread, %.1f s" % (
                          frames, width, height, frames, quality, method,
                          " lossless" if lossless else "", elapsed)}


def measured_traffic(kernel, B, W, H, quality, method):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC
    passes (profiles/r1_pmc_hbm.csv: FETCH_SIZE + WRITE_SIZE in KB, one
    launch of this same default workload), or None for another workload."""
    import csv
    path = os.path.join(HERE, "profiles", "r1_pmc_hbm.csv")
    if not os.path.exists(path) or (B, W, H, quality, method) != (256, 1920, 1080, 75.0, 4):
        return None
    for r in csv.DictReader(open(path)):
        if r["kernel"] == kernel:
            return int(1000 * (float(r["FETCH_SIZE_KB"]) + float(r["WRITE_SIZE_KB"])))
    return None


def shard(rank, frames_per_rank):
    """Frames [first, first + n) owned by `rank`."""
    return rank * frames_per_rank, frames_per_rank


def gather_sizes(sizes, world):
    """All-gather the per-frame encoded sizes of every rank (the only
    data-path collective). Works on any backend (nccl on GPU, gloo in tests)."""
    import torch
    import torch.distributed as dist
    if world == 1:
        return [sizes]
    out = [torch.empty_like(sizes) for _ in range(world)]
    dist.all_gather(out, sizes)
    return out


def max_over_ranks(seconds, world, device):
    import torch
    import torch.distributed as dist
    if world == 1:
        return seconds
    t = torch.tensor([seconds], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def lossless_line(args, world, B, W, H, elapsed, tails, total_bytes):
    """configs[4] line: VP8L encode. Dominant kernel: the L1 transform tile
    kernel (k_vp8l_transform); algorithmic bytes per launch = RGBA read
    (4 B/px) + residual ARGB written (4 B/px) + per-tile modes/multipliers."""
    mp = world * B * W * H * args.steps / 1e6
    steps = len(tails)
    avg = lambda i: sum(t[i] for t in tails) / steps
    tb = 5 if args.method == 4 else (6 if args.method < 4 else 4)
    ntt = ((W + (1 << tb) - 1) >> tb) * ((H + (1 << tb) - 1) >> tb)
    l1_bytes = B * (8 * W * H + 5 * ntt)
    l1_s = avg(7) / 1e6
    achieved = l1_bytes / l1_s / 1e9 if l1_s > 0 else 0.0
    line = {
        "metric": "megapixels/sec encoded (cwebp -lossless -m 4, 1920x1080 batch)",
        "value": round(mp / elapsed, 3),
        "unit": "MP/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8/u32",
        "data": "synthetic syn-v1 RGBA frames generated in HBM (SURVEY.md 8(d))",
        "config": {"workload": "batch of %d %dx%d RGBA frames per GPU, -lossless -q %g -m %d" %
                               (B, W, H, args.quality, args.method),
                   "frames_per_gpu": B, "width": W, "height": H, "quality": args.quality,
                   "method": args.method, "parallelism": "frames sharded %d ways" % world},
        "roofline": {"bound": "hbm", "kernel": "k_vp8l_transform", "achieved": round(achieved, 3),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": None,
                     "k_ms": round(1e3 * l1_s, 3), "algorithmic_bytes_per_launch": l1_bytes},
        "stage_ms": {k: round(avg(i) / 1e3, 3) for k, i in
                     (("transform_analysis", 0), ("host_headers", 1), ("bit_writer", 2),
                      ("d2h", 3), ("riff", 4), ("total", 5), ("k_transform_events", 7),
                      ("k_cache_parse_cluster_events", 6), ("k_write_events", 8))},
        "output_bytes_per_frame": round(total_bytes / (world * B), 1),
    }
    if not args.no_cpu:
        cb = cpu_baseline(W, H, int(args.quality), args.method, args.cpu_seconds, lossless=True)
        if cb:
            line["cpu_baseline"] = cb
    return line


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
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
                    help="config->low_memory (cwebp -low_memory, VP8EncLoop); not the headline config")
    ap.add_argument("--threads", type=int, default=0, help="host tail threads (0 = auto)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--host-input", action="store_true",
                    help="also time one step from host-memory RGBA (PCIe-inclusive)")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)

    import libwebp_amd
    W, H = args.width, args.height
    B = args.batch or (1024 if args.lossless else 256)
    fs = 4 * W * H
    rgba = torch.empty(B * fs, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    first, _ = shard(rank, B)
    libwebp_amd.synth_device(rgba.data_ptr(), W, H, first, B, seed=1, stream=stream)
    torch.cuda.synchronize(dev)
    enc = libwebp_amd.GpuBatch(W, H, B, quality=args.quality, method=args.method, device=local,
                               threads=args.threads, use_sharp_yuv=int(args.sharp_yuv),
                               lossless=int(args.lossless), low_memory=int(args.low_memory))

    def step():
        enc.encode_device(rgba.data_ptr(), B, stream=stream)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)

    for _ in range(args.warmup):
        step()
    barrier()
    t0 = time.perf_counter()
    k3_us, tails = 0.0, []
    for _ in range(args.steps):
        step()
        t = enc.timings()
        k3_us += t[6]
        tails.append(t)
    barrier()
    elapsed = time.perf_counter() - t0
    errs = [enc.error(f) for f in range(B)]
    if any(errs):
        raise RuntimeError("rank %d: frame errors %s" % (rank, sorted(set(errs))))
    sizes = torch.tensor([enc.output_size(f) for f in range(B)], dtype=torch.int64, device=dev)
    ntok = sum(enc.token_count(f) for f in range(B))
    allsizes = gather_sizes(sizes, world)
    elapsed = max_over_ranks(elapsed, world, dev)
    total_bytes = int(sum(int(s.sum().item()) for s in allsizes))

    host_rate = None
    if args.host_input and rank == 0:
        import numpy as np
        host = rgba.view(B, H, W, 4).cpu().numpy()
        t1 = time.perf_counter()
        enc.encode_host(host)
        host_rate = B * W * H / (time.perf_counter() - t1) / 1e6

    if rank != 0:
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return
    if args.lossless:
        print(json.dumps(lossless_line(args, world, B, W, H, elapsed, tails, total_bytes)),
              flush=True)
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        enc.close()
        return
    mp = world * B * W * H * args.steps / 1e6
    value = mp / elapsed
    # K3 (k_encode) roofline: algorithmic bytes per launch = YUV420 planes read
    # (W*H + 2*ceil(W/2)*ceil(H/2) per frame) + 16-bit token stream written +
    # 20 B/MB mode info + the per-frame result block.
    nmb = ((W + 15) // 16) * ((H + 15) // 16)
    yuv = W * H + 2 * ((W + 1) // 2) * ((H + 1) // 2)
    k3_bytes = B * (yuv + 20 * nmb + 1160) + 2 * ntok
    k3_avg_s = k3_us / args.steps / 1e6
    achieved = k3_bytes / k3_avg_s / 1e9 if k3_avg_s > 0 else 0.0
    line = {
        "metric": "megapixels/sec encoded (cwebp -q 75, 1920x1080 batch)",
        "value": round(value, 3),
        "unit": "MP/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8/int32",
        "data": "synthetic syn-v1 RGBA frames generated in HBM (SURVEY.md 8(d))",
        "config": {"workload": "batch of %d %dx%d RGBA frames per GPU, -q %g -m %d%s" %
                               (B, W, H, args.quality, args.method,
                                (" -sharp_yuv" if args.sharp_yuv else "") +
                                (" -low_memory" if args.low_memory else "")),
                   "frames_per_gpu": B, "width": W, "height": H,
                   "quality": args.quality, "method": args.method,
                   "parallelism": "frames sharded %d ways" % world},
        "roofline": {"bound": "hbm", "kernel": "k_encode", "achieved": round(achieved, 3),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 6),
                     "traffic": None if args.sharp_yuv or args.low_memory else
                     measured_traffic("k_encode<3, false, false>", B, W, H, args.quality, args.method),
                     "traffic_source": "profiles/r1_pmc_hbm.csv (rocprofv3 --pmc FETCH_SIZE, "
                                       "WRITE_SIZE passes of this workload; bytes per launch)",
                     "k_encode_ms": round(1e3 * k3_avg_s, 3),
                     "algorithmic_bytes_per_launch": k3_bytes},
        "stage_ms": {k: round(sum(t[i] for t in tails) / len(tails) / 1e3, 3) for k, i in
                     (("import_analysis", 0), ("host_setup", 1), ("rd_tokens", 2),
                      ("d2h", 3), ("host_tail", 4), ("total", 5),
                      ("k_encode_events", 6), ("k_import_analyze_events", 7),
                      ("k_emit_events", 8))},
        "output_bytes_per_frame": round(total_bytes / (world * B), 1),
    }
    if host_rate is not None:
        line["host_input_mps"] = round(host_rate, 3)
    if not args.no_cpu:
        line["cpu_baseline"] = cpu_baseline(W, H, int(args.quality), args.method,
                                            args.cpu_seconds)
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    enc.close()


if __name__ == "__main__":
    main()
