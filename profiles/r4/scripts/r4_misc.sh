#!/bin/bash
# K3 barrier-sleep / lead-priority A/B, the one-rank RCCL leg of bench.py,
# then the K3 trace build at 4 workers with each K3 launch synchronised
# (last: it faulted once). Stops at the first failing step.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=${1:-misc}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
bash tools/ab_libs.sh ${T}_ab main wbs1 lead3; rc=$?; echo "ab rc=$rc" >> $O/steps.log; [ $rc = 0 ] || exit $rc
timeout -k 10 240 python3 bench.py --force-pg --dist-backend nccl --no-cpu --steps 3 --warmup 1 \
  > $O/bench_rccl1.json 2> $O/bench_rccl1.err; rc=$?; echo "rccl rc=$rc" >> $O/steps.log; [ $rc = 0 ] || exit $rc
WEBP_AMD_SYNC_K3=1 WEBP_AMD_LIB=$R/libwebp_amd/libwebp_amd_trace.so timeout -k 10 150 \
  python3 tools/k3_trace.py 1920 1080 256 4 75 $O/k3_trace_256.json > $O/k3_trace_256.log 2>&1
rc=$?; echo "trace rc=$rc" >> $O/steps.log; exit $rc
