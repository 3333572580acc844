set -o pipefail
bash tools/k3x_ab.sh r6ax main late16 &&
WEBP_AMD_LIB=$PWD/libwebp_amd/libwebp_amd_trace.so timeout -k 10 120 python3 tools/k3_trace.py 1920 1080 1 4 75 gpurun_out/r6ax/tr_single_h.json > gpurun_out/r6ax/tr_single_h.log 2>&1
