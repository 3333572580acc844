#!/bin/bash
# Round-5 session 17: the sequential intra-4 path (K3_FORK=0) -- parity subset
# on that library, then K3 A/B: main (fork), seq, round-4's K3.
set -o pipefail
O=gpurun_out/${1:-r5s17}
mkdir -p $O
export PYTHONUNBUFFERED=1
WEBP_AMD_LIB=$(pwd)/libwebp_amd/libwebp_amd_seq.so timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_token_fallbacks.py tests/test_multipass.py tests/test_autofilter.py \
  tests/test_shards.py > $O/tests_seq.log 2>&1 || { echo "tests failed rc=$?"; tail -30 $O/tests_seq.log; exit 1; }
tail -2 $O/tests_seq.log
bash tools/k3_ab.sh ${1:-r5s17}ab main seq r4 || exit 1
