#!/bin/bash
# Lossless (configs[4]) bench line + kernel-time summary, as kept under
# profiles/. Run on the GPU box:  bash tools/profile_lossless.sh <tag>
set -e -o pipefail
TAG=${1:-r1}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_ll_$TAG
mkdir -p $OUT
timeout -k 10 300 python3 $R/bench.py --lossless --steps 3 --warmup 1 > $OUT/bench.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run \
  -- python3 $R/bench.py --lossless --steps 2 --warmup 1 --no-cpu > $OUT/bench_stats.log 2>&1
echo done
