# K4 A/B on one box: the emit / parity tests on the product library, then
# the batch line (1 engine) and one 1080p frame per library variant
set -o pipefail
T=$1; shift; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_emit_gpu.py tests/test_gpu_parity.py -m gpu -x -v --timeout 200 \
  --timeout-method thread > $O/k4_tests.log 2>&1 || exit 1
for r in 1 2; do for v in "$@"; do
  lib=$PWD/libwebp_amd/libwebp_amd_$v.so; [ $v = main ] && lib=$PWD/libwebp_amd/libwebp_amd.so
  WEBP_AMD_LIB=$lib timeout -k 10 120 python3 bench.py --no-cpu --no-host-input --engines 1 --steps 6 --warmup 1 > $O/batch_${v}_$r.json 2> $O/batch_${v}_$r.err || exit 1
  WEBP_AMD_LIB=$lib timeout -k 10 120 python3 bench.py --batch 1 --steps 10 --warmup 2 --no-host-input --no-cpu --engines 1 > $O/single_${v}_$r.json 2> $O/single_${v}_$r.err || exit 1
done; done
