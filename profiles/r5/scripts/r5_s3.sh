#!/bin/bash
# Round-5 session 3: does the session-1 trace+check build (which deadlocked
# at four workers) deadlock again, twice in a row (deterministic for that
# code object)? Then the K3 stage and intra-4 sub-stage splits of the product.
set -o pipefail
O=gpurun_out/r5s3
mkdir -p $O
export PYTHONUNBUFFERED=1
for i in 1 2; do
  WEBP_AMD_LIB=libwebp_amd/libwebp_amd_tc1.so timeout -k 10 200 \
    python -u tools/k3_trace.py 1920 1080 256 4 75 $O/k3_trace_tc1_$i.json > $O/tc1_$i.log 2>&1 || { echo "tc1 run $i failed"; tail -20 $O/tc1_$i.log; exit 1; }
  grep -h k_encode_ms $O/k3_trace_tc1_$i.json
done
WEBP_AMD_LIB=libwebp_amd/libwebp_amd_prof.so timeout -k 10 120 python -u tools/k3_stages.py 1920 1080 256 4 > $O/k3_stages_256.log 2>&1 || exit 1
WEBP_AMD_LIB=libwebp_amd/libwebp_amd_sub.so timeout -k 10 120 python -u tools/k3_stages.py 1920 1080 256 4 > $O/k3_sub_256.log 2>&1 || exit 1
cat $O/k3_stages_256.log $O/k3_sub_256.log | grep -v amdgpu.ids
