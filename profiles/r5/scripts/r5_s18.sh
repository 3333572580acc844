#!/bin/bash
# Round-5 session 18: K3 lineage A/B on one box: round-4's K3, the pre-fork
# K3 of this round (64-bit arena, index checks), the same with the
# barrier / wait changes, main; parity subset on the last variant.
set -o pipefail
O=gpurun_out/${1:-r5s18}
mkdir -p $O
export PYTHONUNBUFFERED=1
WEBP_AMD_LIB=$(pwd)/libwebp_amd/libwebp_amd_c0afb.so timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_token_fallbacks.py tests/test_multipass.py tests/test_autofilter.py \
  tests/test_shards.py > $O/tests_c0afb.log 2>&1 || { echo "tests failed rc=$?"; tail -30 $O/tests_c0afb.log; exit 1; }
tail -2 $O/tests_c0afb.log
bash tools/k3_ab.sh ${1:-r5s18}ab r4 c0af c0afb main || exit 1
