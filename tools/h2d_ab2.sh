#!/bin/bash
# SDMA upload (h2d_sdma.c) against the runtime's copy: host-input bench A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=${1:-h2d2}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 200 python3 -u -m pytest tests/test_host_input.py -m gpu -x -q --timeout 120 \
  --timeout-method thread > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc" >> $O/steps.log
[ $rc = 0 ] || [ $rc = 5 ] || exit $rc
for v in sdma hip sdma hip; do
  LIBWEBP_AMD_H2D=$v timeout -k 10 200 python3 bench.py --no-cpu --steps 4 --warmup 1 > $O/bench_$v.json 2>> $O/bench_$v.err
  rc=$?; echo "h2d $v rc=$rc" >> $O/steps.log; [ $rc = 0 ] || exit $rc
  cp $O/bench_$v.json $O/bench_${v}_$(date +%s).json
done
