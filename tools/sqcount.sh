#!/bin/bash
# SQ issue counters of one bench launch per kernel (separate --pmc passes)
set -e -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/sq${1:-}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU --output-format csv -d $OUT/p1 -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu > $OUT/p1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_WAVES --output-format csv -d $OUT/p2 -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu > $OUT/p2.log 2>&1
echo done
