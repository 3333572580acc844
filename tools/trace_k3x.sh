set -o pipefail
O=gpurun_out/r6am; mkdir -p $O
L=$PWD/libwebp_amd/libwebp_amd_trace.so
WEBP_AMD_LIB=$L timeout -k 10 120 python3 tools/k3_trace.py 1920 1080 1 4 75 $O/tr_single_h.json > $O/tr_single_h.log 2>&1 &&
WEBP_AMD_LIB=$L timeout -k 10 120 python3 tools/k3_trace.py 4096 4096 1 6 90 $O/tr_cfg4_p.json > $O/tr_cfg4_p.log 2>&1
