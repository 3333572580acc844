set -o pipefail
O=gpurun_out/r6ap; mkdir -p $O
for r in 1 2; do for v in main hprio3; do
  lib=$PWD/libwebp_amd/libwebp_amd_$v.so; [ $v = main ] && lib=$PWD/libwebp_amd/libwebp_amd.so
  WEBP_AMD_LIB=$lib timeout -k 10 120 python3 bench.py --batch 1 --steps 10 --warmup 2 --no-host-input --no-cpu --engines 1 > $O/single_${v}_$r.json 2> $O/single_${v}_$r.err || exit 1
  WEBP_AMD_LIB=$lib timeout -k 10 200 python3 bench.py --batch 1 --width 4096 --height 4096 --quality 90 --method 6 --steps 2 --warmup 1 --no-host-input --no-cpu --engines 1 > $O/cfg4_${v}_$r.json 2> $O/cfg4_${v}_$r.err || exit 1
done; done
