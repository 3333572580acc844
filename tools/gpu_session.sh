#!/bin/bash
# One GPU-box session: GPU tests, bench line, K3 stage split, rocprofv3 kernel
# stats, PMC passes (HBM bytes, SQ issue counters) and the PMC calibration.
# Usage (on the box): bash tools/gpu_session.sh <tag> [steps...]
#   steps: tests ltests bench lowmem lossless lab cfg4 lphases lprof lpmc stages stages6 prof pmc sq sq3 calib (default: all but the lossless ones)
set -o pipefail
TAG=${1:-s}; shift
STEPS=${*:-tests bench stages prof pmc sq calib}
START=$(pwd)   # (the smoke step imports __graft_entry__ from here)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/$TAG; mkdir -p $O
cd $R
has() { [[ " $STEPS " == *" $1 "* ]]; }
run() { echo "== $*" >> $O/steps.log; "$@"; local rc=$?; echo "   rc=$rc" >> $O/steps.log; return $rc; }
BENCH="python3 $R/bench.py --no-cpu --no-host-input"
if has boxinfo; then   # CPU share, affinity and clocks of this box
  { echo "cpu.max: $(cat /sys/fs/cgroup/cpu.max 2>/dev/null)"; echo "nproc: $(nproc)";
    python3 -c 'import os; print("affinity:", len(os.sched_getaffinity(0)))';
    rocm-smi --showclocks 2>&1; rocm-smi --showproductname 2>&1 | head -20; } > $O/boxinfo.log 2>&1
fi
if has h2d; then   # H2D / D2H copy rates from pinned host memory (host-input leg)
  run timeout -k 10 120 python3 tools/h2d_probe.py 256 > $O/h2d.json 2> $O/h2d.err || exit 1
  HSA_ENABLE_SDMA=0 run timeout -k 10 120 python3 tools/h2d_probe.py 256 > $O/h2d_nosdma.json \
    2> $O/h2d_nosdma.err || exit 1
fi
if has trace; then   # K3 per-worker wait / stage accounting (the bare trace build: its
  # round-5 fault at 256 frames was found and removed in round 6)
  WEBP_AMD_LIB=$R/libwebp_amd/libwebp_amd_trace.so run timeout -k 10 150 \
    python3 tools/k3_trace.py 1920 1080 256 4 75 $O/k3_trace_256.json > $O/k3_trace_256.log 2>&1 || exit 1
fi
if has budget; then   # the 8-rank host budget on one GPU (quota 16 / 8 ranks = 2 threads) next
  # to the whole-box budget, same box, default line (6 engines, host input); partition 0
  # where the budget puts it (default) and forced to the other side
  run timeout -k 10 300 python3 bench.py --no-cpu > $O/bench_budget16.json 2> $O/bench_budget16.err || exit 1
  WEBP_AMD_CPU_QUOTA=16 LOCAL_WORLD_SIZE=8 run timeout -k 10 300 python3 bench.py --no-cpu \
    > $O/bench_budget2.json 2> $O/bench_budget2.err || exit 1
  WEBP_AMD_P0=gpu run timeout -k 10 300 python3 bench.py --no-cpu > $O/bench_budget16_p0gpu.json \
    2> $O/bench_budget16_p0gpu.err || exit 1
  WEBP_AMD_P0=host WEBP_AMD_CPU_QUOTA=16 LOCAL_WORLD_SIZE=8 run timeout -k 10 300 python3 bench.py \
    --no-cpu > $O/bench_budget2_p0host.json 2> $O/bench_budget2_p0host.err || exit 1
fi
if has p0tests; then   # partition 0 on the device + the core parity tests
  run timeout -k 10 400 python -u -m pytest tests/test_p0_device.py tests/test_gpu_parity.py -m gpu -x -v \
    --timeout 200 --timeout-method thread > $O/gpu_p0tests.log 2>&1 || exit 1
fi
if has trace4; then   # the same for config 4 (one 4096^2 q90 m6 frame, K3X)
  WEBP_AMD_LIB=$R/libwebp_amd/libwebp_amd_trace.so run timeout -k 10 150 \
    python3 tools/k3_trace.py 4096 4096 1 6 90 $O/k3_trace_cfg4.json > $O/k3_trace_cfg4.log 2>&1 || exit 1
fi
if has tests; then
  run timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > $O/gpu_tests.log 2>&1 || exit 1
fi
if has ltests; then   # the lossless GPU tests only
  run timeout -k 10 400 python -u -m pytest tests/test_vp8l.py -m gpu -x -v --timeout 120 \
    --timeout-method thread > $O/gpu_ltests.log 2>&1 || exit 1
fi
if has bench; then
  run timeout -k 10 400 python3 bench.py --steps 5 --warmup 2 > $O/bench.json 2> $O/bench.err || exit 1
fi
if has engab; then   # encoder instances per GPU: 3 (9 steps) vs 4 (12 steps), host-input line
  for i in 1 2; do
    run timeout -k 10 300 python3 bench.py --no-cpu --steps 9 --warmup 2 --engines 3 \
      > $O/eng3_$i.json 2> $O/eng3_$i.err || exit 1
    run timeout -k 10 300 python3 bench.py --no-cpu --steps 12 --warmup 2 --engines 4 \
      > $O/eng4_$i.json 2> $O/eng4_$i.err || exit 1
  done
fi
if has h2dab; then   # runtime copies vs SDMA (LIBWEBP_AMD_H2D=hip), one and three engines
  LIBWEBP_AMD_H2D=hip run timeout -k 10 300 python3 bench.py --no-cpu --steps 3 --warmup 1 \
    > $O/h2dab_hip.json 2> $O/h2dab_hip.err || exit 1
  run timeout -k 10 300 python3 bench.py --no-cpu --steps 3 --warmup 1 --engines 1 \
    > $O/h2dab_e1.json 2> $O/h2dab_e1.err || exit 1
fi
if has bench0; then   # the line exactly as the driver's default run makes it
  run timeout -k 10 400 python3 bench.py > $O/bench0.json 2> $O/bench0.err || exit 1
fi
if has lowmem; then   # low_memory (K3 once per pass, tokens re-derived)
  run timeout -k 10 400 python3 bench.py --low-memory --steps 3 --warmup 1 --no-cpu > $O/bench_lowmem.json \
    2> $O/bench_lowmem.err || exit 1
fi
if has lossless; then
  run timeout -k 10 400 python3 bench.py --lossless --steps 6 --warmup 1 > $O/bench_lossless.json \
    2> $O/bench_lossless.err || exit 1
fi
if has lab; then   # lossless encoder instances: 2 vs 3 (balanced step counts)
  for i in 1 2; do
    run timeout -k 10 300 $BENCH --lossless --engines 2 --steps 4 --warmup 1 > $O/lab_e2_$i.json \
      2> $O/lab_e2_$i.err || exit 1
    run timeout -k 10 300 $BENCH --lossless --engines 3 --steps 6 --warmup 1 > $O/lab_e3_$i.json \
      2> $O/lab_e3_$i.err || exit 1
  done
fi
if has cfg4; then   # config 4 (one 4096^2 q90 m6 frame, K3X) and one 1080p frame
  run timeout -k 10 300 python3 bench.py --batch 1 --width 4096 --height 4096 --quality 90 --method 6 \
    --steps 2 --warmup 1 --no-host-input --cpu-seconds 10 --engines 1 > $O/bench_cfg4.json \
    2> $O/bench_cfg4.err || exit 1
  run timeout -k 10 300 python3 bench.py --batch 1 --steps 10 --warmup 2 --no-host-input --no-cpu \
    --engines 1 > $O/bench_1080p_single.json 2> $O/bench_1080p_single.err || exit 1
fi
if has k3xab; then   # K3X with 1 worker per workgroup (WEBP_AMD_K3X_NW=1) against 2: its
  # parity tests first, then config 4 and one 1080p frame each way
  WEBP_AMD_K3X_NW=1 run timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_concurrency.py \
    tests/test_token_fallbacks.py tests/test_early_fold.py -m gpu -x -v --timeout 200 --timeout-method thread \
    > $O/k3x1_tests.log 2>&1 || exit 1
  for NWX in 2 1; do
    WEBP_AMD_K3X_NW=$NWX run timeout -k 10 300 python3 bench.py --batch 1 --width 4096 --height 4096 --quality 90 \
      --method 6 --steps 2 --warmup 1 --no-host-input --no-cpu --engines 1 > $O/cfg4_nw$NWX.json \
      2> $O/cfg4_nw$NWX.err || exit 1
    WEBP_AMD_K3X_NW=$NWX run timeout -k 10 300 python3 bench.py --batch 1 --steps 10 --warmup 2 --no-host-input \
      --no-cpu --engines 1 > $O/single_nw$NWX.json 2> $O/single_nw$NWX.err || exit 1
  done
fi
if has k3xhp; then   # K3X helper pairs (WEBP_AMD_K3X_NW=h) against one worker: parity
  # tests first, then config 4 and one 1080p frame each way
  WEBP_AMD_K3X_NW=h run timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_concurrency.py \
    tests/test_token_fallbacks.py tests/test_early_fold.py -m gpu -x -v --timeout 200 --timeout-method thread \
    > $O/k3xh_tests.log 2>&1 || exit 1
  for NWX in h 1; do
    WEBP_AMD_K3X_NW=$NWX run timeout -k 10 300 python3 bench.py --batch 1 --width 4096 --height 4096 --quality 90 \
      --method 6 --steps 2 --warmup 1 --no-host-input --no-cpu --engines 1 > $O/cfg4_nw$NWX.json \
      2> $O/cfg4_nw$NWX.err || exit 1
    WEBP_AMD_K3X_NW=$NWX run timeout -k 10 300 python3 bench.py --batch 1 --steps 10 --warmup 2 --no-host-input \
      --no-cpu --engines 1 > $O/single_nw$NWX.json 2> $O/single_nw$NWX.err || exit 1
  done
fi
if has k3xp; then   # K3X helper pairs with an intra-4 partner (WEBP_AMD_K3X_NW=p) against the
  # helper pairs (default): parity tests first, then config 4 and one 1080p frame each way
  WEBP_AMD_K3X_NW=p run timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_concurrency.py \
    tests/test_token_fallbacks.py tests/test_early_fold.py tests/test_progress.py -m gpu -x -v --timeout 200 \
    --timeout-method thread > $O/k3xp_tests.log 2>&1 || exit 1
  for NWX in p h; do
    WEBP_AMD_K3X_NW=$NWX run timeout -k 10 300 python3 bench.py --batch 1 --width 4096 --height 4096 --quality 90 \
      --method 6 --steps 2 --warmup 1 --no-host-input --no-cpu --engines 1 > $O/cfg4_nw$NWX.json \
      2> $O/cfg4_nw$NWX.err || exit 1
    WEBP_AMD_K3X_NW=$NWX run timeout -k 10 300 python3 bench.py --batch 1 --steps 10 --warmup 2 --no-host-input \
      --no-cpu --engines 1 > $O/single_nw$NWX.json 2> $O/single_nw$NWX.err || exit 1
  done
fi
if has k3xhw; then   # K3X one row worker with the hardware barrier (WEBP_AMD_K3X_NW=1) against
  # the helper pairs (default): parity tests first, then config 4 and one 1080p frame each way
  WEBP_AMD_K3X_NW=1 run timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_concurrency.py \
    tests/test_token_fallbacks.py tests/test_early_fold.py tests/test_progress.py -m gpu -x -v --timeout 200 \
    --timeout-method thread > $O/k3x1hw_tests.log 2>&1 || exit 1
  for NWX in 1 h; do
    WEBP_AMD_K3X_NW=$NWX run timeout -k 10 300 python3 bench.py --batch 1 --width 4096 --height 4096 --quality 90 \
      --method 6 --steps 2 --warmup 1 --no-host-input --no-cpu --engines 1 > $O/cfg4_nw$NWX.json \
      2> $O/cfg4_nw$NWX.err || exit 1
    WEBP_AMD_K3X_NW=$NWX run timeout -k 10 300 python3 bench.py --batch 1 --steps 10 --warmup 2 --no-host-input \
      --no-cpu --engines 1 > $O/single_nw$NWX.json 2> $O/single_nw$NWX.err || exit 1
  done
fi
if has emittests; then   # K4 alone (compact and row streams)
  run timeout -k 10 300 python -u -m pytest tests/test_emit_gpu.py -m gpu -x -v --timeout 200 \
    --timeout-method thread > $O/emit_tests.log 2>&1 || exit 1
fi
if has lprof; then
  (cd /tmp && TMPDIR=/tmp run timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $O/lstats -o run -- python3 $R/bench.py --lossless --no-cpu --no-host-input --steps 2 \
    --warmup 1 > $O/lprof.log 2>&1) || exit 1
fi
if has lphases; then   # L1a / L1 phase cycles (diagnostic build)
  WEBP_AMD_LIB=$R/libwebp_amd/libwebp_amd_prof.so run timeout -k 10 150 \
    python3 tools/vp8l_phases.py 1920 1080 256 4 > $O/vp8l_phases.log 2>&1 || exit 1
fi
if has dptime; then   # lossless text frames (the shortest-path parse on every frame)
  (cd /tmp && TMPDIR=/tmp run timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $O/dpstats -o run -- python3 $R/tools/dp_time.py 64 > $O/dptime.json 2> $O/dptime.err) || exit 1
fi
if has lprof1; then   # the lossless kernels one instance at a time (solo durations)
  (cd /tmp && TMPDIR=/tmp run timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $O/lstats1 -o run -- python3 $R/bench.py --lossless --no-cpu --no-host-input --steps 2 \
    --warmup 1 --engines 1 > $O/lprof1.log 2>&1) || exit 1
fi
if has prof1; then   # the lossy kernels one instance at a time
  (cd /tmp && TMPDIR=/tmp run timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $O/stats1 -o run -- python3 $R/bench.py --no-cpu --no-host-input --steps 2 \
    --warmup 1 --engines 1 > $O/prof1.log 2>&1) || exit 1
fi
if has stages; then
  for B in 256 1; do
    WEBP_AMD_LIB=$R/libwebp_amd/libwebp_amd_prof.so run timeout -k 10 150 \
      python3 tools/k3_stages.py 1920 1080 $B 4 > $O/stages_$B.log 2>&1 || exit 1
  done
fi
if has stages6; then   # m6 (config 4's method) stage split at 1080p, and the intra-4 sub-stages
  WEBP_AMD_LIB=$R/libwebp_amd/libwebp_amd_prof.so run timeout -k 10 200 \
    python3 tools/k3_stages.py 1920 1080 256 6 > $O/stages6_256.log 2>&1 || exit 1
  WEBP_AMD_LIB=$R/libwebp_amd/libwebp_amd_sub.so run timeout -k 10 200 \
    python3 tools/k3_stages.py 1920 1080 256 6 > $O/sub6_256.log 2>&1 || exit 1
fi
cd /tmp && export TMPDIR=/tmp
if has prof; then
  run timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run \
    -- $BENCH --steps 2 --warmup 1 > $O/prof.log 2>&1 || exit 1
fi
if has xprof; then   # one 1080p frame and config 4 (K3X): kernel stats
  run timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/xstats -o run \
    -- python3 $R/bench.py --batch 1 --steps 10 --warmup 2 --no-host-input --no-cpu --engines 1 \
    > $O/xprof.log 2>&1 || exit 1
  run timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/x4stats -o run \
    -- python3 $R/bench.py --batch 1 --width 4096 --height 4096 --quality 90 --method 6 --steps 2 \
    --warmup 1 --no-host-input --no-cpu --engines 1 > $O/x4prof.log 2>&1 || exit 1
fi
if has smoke; then
  (cd $START && run timeout -k 10 300 python3 -c 'import __graft_entry__ as g; g.smoke()') > $O/smoke.log 2>&1 || exit 1
fi
if has hprof; then   # host-input bench (SDMA upload): kernel timeline
  run timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/hstats -o run \
    -- python3 $R/bench.py --no-cpu --steps 3 --warmup 1 > $O/hprof.log 2>&1 || exit 1
fi
if has copytrace; then   # host-input bench: kernels and memory copies (SDMA or blit kernel)
  run timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv \
    -d $O/ctrace -o run -- python3 $R/bench.py --no-cpu --steps 2 --warmup 1 > $O/ctrace.log 2>&1 || exit 1
fi
if has pmc; then
  for C in FETCH_SIZE WRITE_SIZE; do
    run timeout -s KILL 200 rocprofv3 --pmc $C --output-format csv -d $O/pmc_$C -o run \
      -- $BENCH --steps 1 --warmup 0 > $O/pmc_$C.log 2>&1 || exit 1
  done
fi
if has sq; then
  run timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU --output-format csv -d $O/sq1 -o run \
    -- $BENCH --steps 1 --warmup 0 > $O/sq1.log 2>&1 || exit 1
  run timeout -s KILL 200 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS \
    SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_WAVES --output-format csv -d $O/sq2 -o run \
    -- $BENCH --steps 1 --warmup 0 > $O/sq2.log 2>&1 || exit 1
fi
if has lpmc; then   # HBM bytes of the lossless kernels (bench.py --lossless, one step)
  for C in FETCH_SIZE WRITE_SIZE; do
    run timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d $O/lpmc/pmc_$C -o run \
      -- python3 $R/bench.py --lossless --no-cpu --no-host-input --steps 1 --warmup 0 \
      > $O/lpmc_$C.log 2>&1 || exit 1
  done
fi
if has sq3; then   # VALU lane utilisation (thread-cycles per VALU cycle); last: a counter
  run timeout -s KILL 120 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU \
    --output-format csv -d $O/sq3 -o run -- $BENCH --steps 1 --warmup 0 > $O/sq3.log 2>&1 || exit 1
fi
if has calib; then
  for C in FETCH_SIZE WRITE_SIZE; do
    run timeout -s KILL 60 rocprofv3 --pmc $C --output-format csv -d $O/calib_$C -o run \
      -- $R/tools/bin/pmc_calib > $O/calib_$C.log 2>&1 || exit 1
  done
fi
# (last: these may fault the GPU, and nothing runs after a fault)
cd $R
if has tracebare; then   # the bare trace build (-DK3_TRACE) at 256 frames; the runtime's
  # fault report (address, reason) with AMD_LOG_LEVEL=1. Last step: it may fault.
  AMD_LOG_LEVEL=1 WEBP_AMD_FAULT_REPORT=1 WEBP_AMD_LIB=$R/libwebp_amd/libwebp_amd_trace.so run timeout -k 10 150 \
    python3 tools/k3_trace.py 1920 1080 256 4 75 $O/k3_trace_bare_256.json > $O/k3_trace_bare_256.log 2>&1 || exit 1
fi
if has tracediff; then   # bare trace builds of other K3 sources (make ab AB=<name>
  # ABSRC=... ABFLAGS=-DK3_TRACE), in the order of $TRACE_ABS; stops at the first failure
  for A in $TRACE_ABS; do
    AMD_LOG_LEVEL=1 WEBP_AMD_FAULT_REPORT=1 WEBP_AMD_LIB=$R/libwebp_amd/libwebp_amd_$A.so run timeout -k 10 150 \
      python3 tools/k3_trace.py 1920 1080 256 4 75 $O/k3_trace_$A.json > $O/k3_trace_$A.log 2>&1 || exit 1
  done
fi
echo "session $TAG done" >> $O/steps.log
