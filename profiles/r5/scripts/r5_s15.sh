#!/bin/bash
# Round-5 session 15: the epoch-priority build failed with an exhausted token
# arena: once more, then with the index checks; round-4's K3 against main.
O=gpurun_out/${1:-r5s15}
mkdir -p $O
export PYTHONUNBUFFERED=1
for v in eprio eprioc; do
  WEBP_AMD_LIB=libwebp_amd/libwebp_amd_$v.so timeout -k 10 150 python -u tools/k3_hang.py 1920 1080 256 4 > $O/$v.log 2>&1
  rc=$?; echo "$v rc=$rc"; grep -v amdgpu.ids $O/$v.log | head -20
  case $rc in 0|1) ;; *) exit $rc;; esac
done
bash tools/k3_ab.sh ${1:-r5s15}ab main r4 || exit 1
