set -o pipefail
mkdir -p gpurun_out/x1
export WEBP_AMD_K3X=1
timeout -k 10 120 python3 -u tools/k3x_time.py 1920 1080 1 75 4 3 > gpurun_out/x1/t1080_x.json 2> gpurun_out/x1/t1080_x.err || exit 1
timeout -k 10 120 python3 -u tools/k3x_time.py 512 512 4 75 4 3 > gpurun_out/x1/t512_x.json 2> gpurun_out/x1/t512_x.err || exit 1
WEBP_AMD_K3X=0 timeout -k 10 120 python3 -u tools/k3x_time.py 1920 1080 1 75 4 3 > gpurun_out/x1/t1080_0.json 2> gpurun_out/x1/t1080_0.err || exit 1
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/x1/gpu_tests.log 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/k3x_time.py 4096 4096 1 90 6 1 > gpurun_out/x1/t4096_x.json 2> gpurun_out/x1/t4096_x.err || exit 1
