set -o pipefail
O=gpurun_out/r6au; mkdir -p $O
for r in 1 2; do for v in p h; do
  WEBP_AMD_K3X_NW=$v timeout -k 10 120 python3 bench.py --batch 1 --steps 10 --warmup 2 --no-host-input --no-cpu --engines 1 > $O/single_nw${v}_$r.json 2> $O/single_nw${v}_$r.err || exit 1
  WEBP_AMD_K3X_NW=$v timeout -k 10 200 python3 bench.py --batch 1 --width 4096 --height 4096 --quality 90 --method 6 --steps 2 --warmup 1 --no-host-input --no-cpu --engines 1 > $O/cfg4_nw${v}_$r.json 2> $O/cfg4_nw${v}_$r.err || exit 1
done; done
