# K3X per-worker accounting (trace build) and the main worker's intra-4
# sub-stage split (SUBPROF build), one 1080p q75 m4 picture
set -o pipefail
O=gpurun_out/${1:-r6at}; mkdir -p $O
WEBP_AMD_LIB=$PWD/libwebp_amd/libwebp_amd_trace.so timeout -k 10 120 python3 tools/k3_trace.py 1920 1080 1 4 75 $O/tr_single_h.json > $O/tr_single_h.log 2>&1 &&
WEBP_AMD_LIB=$PWD/libwebp_amd/libwebp_amd_sub.so timeout -k 10 120 python3 tools/k3x_sub.py 1920 1080 4 75 > $O/sub_single.log 2>&1
