#!/bin/bash
# Round-5 session 1 on the GPU box: the token-buffer fallbacks and the parity
# suite on the product library, the 4-worker trace build with index checks on
# the 256 x 1080p batch, then one default bench line.
set -o pipefail
O=gpurun_out/r5s1
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_token_fallbacks.py tests/test_gpu_parity.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
WEBP_AMD_LIB=libwebp_amd/libwebp_amd_tracecheck.so timeout -k 10 300 \
  python -u tools/k3_trace.py 1920 1080 256 4 75 $O/k3_trace_nw4.json > $O/tracecheck.log 2>&1 || { echo "tracecheck failed"; tail -20 $O/tracecheck.log; exit 1; }
grep K3_CHECK $O/tracecheck.log
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
tail -c 1500 $O/bench.json
