#!/bin/bash
# Round-5 session 34: the trace build with its replay counter, row-wait
# counter and reset branch-free, at 256 x 1080p; then main vs fold inlined.
set -o pipefail
O=gpurun_out/${1:-r5s34}
mkdir -p $O
WEBP_AMD_LIB=$(pwd)/libwebp_amd/libwebp_amd_trace.so timeout -k 10 50 python3 tools/k3_trace.py 1920 1080 256 4 75 \
  $O/k3_trace_256.json > $O/k3_trace_256.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc = 0 ] || { tail -3 $O/k3_trace_256.log; exit $rc; }
python3 -c "import json;d=json.load(open('$O/k3_trace_256.json'));print('trace', d['k_encode_ms'], d['share_of_worker_cycles'])"
bash tools/k3_ab.sh ${1:-r5s34}ab main inl || exit 1
