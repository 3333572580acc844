#!/bin/bash
# 4-worker K3 (diagnostic build, WEBP_AMD_K3=4) on the m3/m4 parity cases,
# each K3 launch synchronised (a fault names its launch), then the solo
# bench against the default 3-worker kernel of the same library. Stops at
# the first failing step.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=${1:-nw4}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
export WEBP_AMD_LIB=$R/libwebp_amd/libwebp_amd_diag.so WEBP_AMD_K3X=0
WEBP_AMD_K3=4 WEBP_AMD_SYNC_K3=1 timeout -k 10 240 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
  -k "m4 or m3 or m2 or kat_1080p or kat_512 or committed" --timeout 120 --timeout-method thread > $O/nw4_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $O/steps.log; [ $rc = 0 ] || exit $rc
for v in 4 0; do
  WEBP_AMD_K3=$v timeout -k 10 200 python3 bench.py --no-cpu --no-host-input --engines 1 --steps 3 --warmup 1 \
    > $O/bench_k3_$v.json 2> $O/bench_k3_$v.err
  rc=$?; echo "bench $v rc=$rc" >> $O/steps.log; [ $rc = 0 ] || exit $rc
done
