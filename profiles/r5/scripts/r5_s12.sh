#!/bin/bash
# Round-5 session 12: barriers / waits without compiler-visible lane masks
# (asm arrival, scalar polls): parity subset, same-box A/B against the last
# commit's K3, then the stage split (the build that stalled before), the
# intra-4 split and the 4-worker trace.
set -o pipefail
O=gpurun_out/${1:-r5s12}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_token_fallbacks.py tests/test_multipass.py tests/test_autofilter.py \
  tests/test_shards.py > $O/tests.log 2>&1 || { echo "tests failed rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/k3_ab.sh ${1:-r5s12}ab main prev || exit 1
WEBP_AMD_LIB=libwebp_amd/libwebp_amd_prof.so timeout -k 10 120 python -u tools/k3_stages.py 1920 1080 256 4 > $O/k3_stages_256.log 2>&1
rc=$?; echo "stages rc=$rc"; grep -v amdgpu.ids $O/k3_stages_256.log; [ $rc = 0 ] || exit $rc
WEBP_AMD_LIB=libwebp_amd/libwebp_amd_sub.so timeout -k 10 120 python -u tools/k3_stages.py 1920 1080 256 4 > $O/k3_sub_256.log 2>&1
rc=$?; echo "sub rc=$rc"; grep -v amdgpu.ids $O/k3_sub_256.log; [ $rc = 0 ] || exit $rc
WEBP_AMD_LIB=libwebp_amd/libwebp_amd_trace.so timeout -k 10 120 python -u tools/k3_trace.py 1920 1080 256 4 75 $O/k3_trace.json > $O/k3_trace.log 2>&1
rc=$?; echo "trace rc=$rc"; python3 -c "import json;d=json.load(open('$O/k3_trace.json'));print(d['k_encode_ms'], d['share_of_worker_cycles'])"; exit $rc
