#!/bin/bash
# Round-5 session 32: the trace build with fold_mbs inlined (the hang came
# with fold_mbs<8> out of line, b59c671) at 256 x 1080p, then batch K3 A/B
# main vs inlined.
set -o pipefail
O=gpurun_out/${1:-r5s32}
mkdir -p $O
WEBP_AMD_LIB=$(pwd)/libwebp_amd/libwebp_amd_trinl.so timeout -k 10 50 python3 tools/k3_trace.py 1920 1080 256 4 75 \
  $O/tr_inl.json > $O/tr_inl.log 2>&1
rc=$?; echo "trinl rc=$rc"; [ $rc = 0 ] || { tail -3 $O/tr_inl.log; exit $rc; }
python3 -c "import json;d=json.load(open('$O/tr_inl.json'));print('trinl', d['k_encode_ms'], d['share_of_worker_cycles'])"
bash tools/k3_ab.sh ${1:-r5s32}ab main inl || exit 1
