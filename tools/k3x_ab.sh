# K3X check on one box: the K3X parity tests, then config 4 and one 1080p
# frame per library variant (usage: bash tools/k3x_ab.sh <tag> <variant>...;
# "main" = libwebp_amd.so)
set -o pipefail
T=$1; shift; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_concurrency.py tests/test_token_fallbacks.py \
  tests/test_early_fold.py tests/test_progress.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/k3x_tests.log 2>&1 || exit 1
for r in 1 2; do for v in "$@"; do
  lib=$PWD/libwebp_amd/libwebp_amd_$v.so; [ $v = main ] && lib=$PWD/libwebp_amd/libwebp_amd.so
  WEBP_AMD_LIB=$lib timeout -k 10 120 python3 bench.py --batch 1 --steps 10 --warmup 2 --no-host-input --no-cpu --engines 1 > $O/single_${v}_$r.json 2> $O/single_${v}_$r.err || exit 1
  WEBP_AMD_LIB=$lib timeout -k 10 200 python3 bench.py --batch 1 --width 4096 --height 4096 --quality 90 --method 6 --steps 2 --warmup 1 --no-host-input --no-cpu --engines 1 > $O/cfg4_${v}_$r.json 2> $O/cfg4_${v}_$r.err || exit 1
done; done
if [ -n "$K3X_NWP" ]; then   # the partner form on one 1080p frame, the product library
  for r in 1 2; do
    WEBP_AMD_K3X_NW=p timeout -k 10 120 python3 bench.py --batch 1 --steps 10 --warmup 2 --no-host-input --no-cpu --engines 1 > $O/single_nwp_$r.json 2> $O/single_nwp_$r.err || exit 1
  done
fi
