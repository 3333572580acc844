#!/bin/bash
# Round-5 session 13: intra-4 loads one sub-block ahead; A/B against the last
# commit and an epoch-boundary priority variant; stage splits.
set -o pipefail
O=gpurun_out/${1:-r5s13}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_token_fallbacks.py tests/test_multipass.py tests/test_autofilter.py \
  tests/test_shards.py > $O/tests.log 2>&1 || { echo "tests failed rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/k3_ab.sh ${1:-r5s13}ab main prev eprio || exit 1
WEBP_AMD_LIB=libwebp_amd/libwebp_amd_prof.so timeout -k 10 120 python -u tools/k3_stages.py 1920 1080 256 4 > $O/k3_stages_256.log 2>&1
rc=$?; echo "stages rc=$rc"; grep -v amdgpu.ids $O/k3_stages_256.log; [ $rc = 0 ] || exit $rc
WEBP_AMD_LIB=libwebp_amd/libwebp_amd_sub.so timeout -k 10 120 python -u tools/k3_stages.py 1920 1080 256 4 > $O/k3_sub_256.log 2>&1
rc=$?; echo "sub rc=$rc"; grep -v amdgpu.ids $O/k3_sub_256.log; exit $rc
