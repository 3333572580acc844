#!/bin/bash
# Kernel-time summary + HBM counters of the default bench workload, as kept
# under profiles/. Run on the GPU box:  bash tools/profile_round.sh <tag>
set -e -o pipefail
TAG=${1:-r1}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run \
  -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu > $OUT/bench_stats.log 2>&1
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $C --output-format csv -d $OUT/pmc_$C -o run \
    -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu > $OUT/bench_$C.log 2>&1
done
echo done
