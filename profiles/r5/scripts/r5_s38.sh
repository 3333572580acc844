#!/bin/bash
# Round-5 session 38 (votes read after the next MB): folds of a row's pending deltas before their 16-bit
# fields could wrap: parity of the build that folds at a tiny threshold
# (every 16-MB column once any slot has 64 pending tokens) and of the
# product build; batch K3 A/B against the build without the check.
set -o pipefail
O=gpurun_out/${1:-r5s38}
mkdir -p $O
export PYTHONUNBUFFERED=1
WEBP_AMD_LIB=$(pwd)/libwebp_amd/libwebp_amd_dfull.so timeout -k 10 600 python -u -m pytest -x -v --timeout 300 \
  --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_token_fallbacks.py tests/test_multipass.py \
  tests/test_shards.py > $O/tests_dfull.log 2>&1 || { echo "dfull tests failed rc=$?"; tail -30 $O/tests_dfull.log; exit 1; }
tail -1 $O/tests_dfull.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
  > $O/tests.log 2>&1 || { echo "tests failed rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/k3_ab.sh ${1:-r5s38}ab main nodfull || exit 1
