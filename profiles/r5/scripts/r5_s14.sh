#!/bin/bash
# Round-5 session 14: the reverted intra-4 loop against the last commit and the
# epoch-boundary priority variant; m6 stage split at 1080p.
set -o pipefail
O=gpurun_out/${1:-r5s14}
mkdir -p $O
export PYTHONUNBUFFERED=1
bash tools/k3_ab.sh ${1:-r5s14}ab main prev eprio || exit 1
WEBP_AMD_LIB=libwebp_amd/libwebp_amd_prof.so timeout -k 10 200 python -u tools/k3_stages.py 1920 1080 256 6 > $O/k3_stages_256_m6.log 2>&1
rc=$?; echo "stages m6 rc=$rc"; grep -v amdgpu.ids $O/k3_stages_256_m6.log; [ $rc = 0 ] || exit $rc
WEBP_AMD_LIB=libwebp_amd/libwebp_amd_sub.so timeout -k 10 200 python -u tools/k3_stages.py 1920 1080 256 6 > $O/k3_sub_256_m6.log 2>&1
rc=$?; echo "sub m6 rc=$rc"; grep -v amdgpu.ids $O/k3_sub_256_m6.log; exit $rc
