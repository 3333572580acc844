#!/bin/bash
# Round-5 session 35: the trace build with the batch replay at 4 chunks per
# step (as before b59c671) at 256 x 1080p; batch K3 A/B main (8) vs rd4.
set -o pipefail
O=gpurun_out/${1:-r5s35}
mkdir -p $O
WEBP_AMD_LIB=$(pwd)/libwebp_amd/libwebp_amd_trrd4.so timeout -k 10 50 python3 tools/k3_trace.py 1920 1080 256 4 75 \
  $O/k3_trace_256.json > $O/k3_trace_256.log 2>&1
rc=$?; echo "trrd4 rc=$rc"; [ $rc = 0 ] || { tail -3 $O/k3_trace_256.log; exit $rc; }
python3 -c "import json;d=json.load(open('$O/k3_trace_256.json'));print('trace', d['k_encode_ms'], d['share_of_worker_cycles'])"
bash tools/k3_ab.sh ${1:-r5s35}ab main rd4 || exit 1
