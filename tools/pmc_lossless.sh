#!/bin/bash
# SQ counters of the lossless kernels (one pass, 8 SQ slots). GPU box only.
set -e -o pipefail
TAG=${1:-r1}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_ll_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $OUT/sq -o run \
  -- python3 $R/bench.py --lossless --batch 256 --steps 1 --warmup 0 --no-cpu > $OUT/bench.log 2>&1
echo done
