#!/bin/bash
# Double-buffered host upload (WebPGpuBatchEncodeRGBAHostPrefetch): GPU tests,
# then the default line with / without it and with 5 instances, two rounds.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/$1; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests/test_host_prefetch.py tests/test_host_input.py -m gpu -x -v \
  --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --no-cpu > $O/pf4_$i.json 2> $O/pf4_$i.err || exit 1
  timeout -k 10 300 python3 bench.py --no-cpu --no-prefetch > $O/np4_$i.json 2> $O/np4_$i.err || exit 1
  timeout -k 10 300 python3 bench.py --no-cpu --engines 5 --steps 15 > $O/pf5_$i.json 2> $O/pf5_$i.err || exit 1
done
echo done > $O/done
