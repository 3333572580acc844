#!/bin/bash
# Round-2 measurement session on the GPU box: bench lines (headline, config 4,
# single 1080p WebPEncode-sized batch, lossless), rocprofv3 kernel stats of the headline
# bench, FETCH_SIZE / WRITE_SIZE PMC passes (one counter per pass).
# usage (on the box): bash tools/gpu_profile_r2.sh TAG
set -o pipefail
TAG=${1:-p}
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/$TAG; mkdir -p $O
cd $R
run() { echo "== $*" >> $O/steps.log; "$@"; local rc=$?; echo "   rc=$rc" >> $O/steps.log; return $rc; }
run timeout -k 10 400 python3 bench.py --steps 5 --warmup 2 > $O/bench.json 2> $O/bench.err || exit 1
run timeout -k 10 300 python3 bench.py --batch 1 --width 4096 --height 4096 --quality 90 --method 6 \
  --steps 2 --warmup 1 --no-host-input --cpu-seconds 10 --engines 1 > $O/bench_cfg4.json 2> $O/bench_cfg4.err || exit 1
run timeout -k 10 300 python3 bench.py --batch 1 --steps 10 --warmup 2 --no-host-input --no-cpu \
  --engines 1 > $O/bench_1080p_single.json 2> $O/bench_1080p_single.err || exit 1
run timeout -k 10 300 python3 bench.py --lossless --steps 4 --warmup 1 --no-host-input --no-cpu \
  > $O/bench_lossless.json 2> $O/bench_lossless.err || exit 1
BENCH="python3 $R/bench.py --no-cpu --no-host-input"
cd /tmp && export TMPDIR=/tmp
run timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run \
  -- $BENCH --steps 2 --warmup 1 > $O/prof.log 2>&1 || exit 1
for C in FETCH_SIZE WRITE_SIZE; do
  run timeout -s KILL 200 rocprofv3 --pmc $C --output-format csv -d $O/pmc_$C -o run \
    -- $BENCH --steps 1 --warmup 0 > $O/pmc_$C.log 2>&1 || exit 1
done
echo "session $TAG done" >> $O/steps.log
