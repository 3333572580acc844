#!/bin/bash
# Round-5 session 9: same-box K3 A/B of the working tree against the last
# commit's K3 (base), then the coarse stage split of the working tree.
set -o pipefail
O=gpurun_out/${1:-r5s9}
mkdir -p $O
export PYTHONUNBUFFERED=1
bash tools/k3_ab.sh ${1:-r5s9}ab main base nopf f16 || exit 1
WEBP_AMD_LIB=libwebp_amd/libwebp_amd_prof.so timeout -k 10 120 python -u tools/k3_stages.py 1920 1080 256 4 > $O/k3_stages_256.log 2>&1
rc=$?; echo "stages rc=$rc"; cat $O/k3_stages_256.log; exit $rc
