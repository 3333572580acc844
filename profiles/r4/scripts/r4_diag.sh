#!/bin/bash
# round-4 diagnosis session: trellis self-test (diagnostic build), the GPU
# suite without -x (failures listed, not fatal), then the K3 A/B bench.
# Stops at the first step that times out or crashes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=${1:-r4d}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
ok() { local rc=$1; [ "$rc" = 0 ] || [ "$rc" = 1 ]; }
WEBP_AMD_LIB=$R/libwebp_amd/libwebp_amd_trace.so timeout -k 10 60 python3 tools/trellis_selftest.py 4096 \
  > $O/trellis.json 2> $O/trellis.err; rc=$?; echo "trellis rc=$rc" >> $O/steps.log; ok $rc || exit $rc
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q -rf --maxfail=60 --timeout 120 --timeout-method thread \
  > $O/gpu_tests.log 2>&1; rc=$?; echo "tests rc=$rc" >> $O/steps.log; ok $rc || exit $rc
bash tools/ab_libs.sh ${T}_ab main base; rc=$?; echo "ab rc=$rc" >> $O/steps.log
exit $rc
