#!/bin/bash
# Round-5 session 26: replay depth A/B: batch K3 (4 vs 8 chunks per step),
# config 4 K3X (16 vs 32 vs 8).
set -o pipefail
O=gpurun_out/${1:-r5s26}
mkdir -p $O
bash tools/k3_ab.sh ${1:-r5s26}ab main rdb8 || exit 1
for round in 1 2; do
  for v in main rdx32 rdx8; do
    lib=$(pwd)/libwebp_amd/libwebp_amd_$v.so; [ $v = main ] && lib=$(pwd)/libwebp_amd/libwebp_amd.so
    WEBP_AMD_LIB=$lib timeout -k 10 200 python3 bench.py --batch 1 --width 4096 --height 4096 --quality 90 --method 6 \
      --steps 2 --warmup 1 --no-host-input --no-cpu --engines 1 > $O/cfg4_${v}_$round.json 2> $O/cfg4_${v}_$round.err || exit 1
    python3 -c "import json;d=json.loads(open('$O/cfg4_${v}_$round.json').read().strip().splitlines()[-1]);print('cfg4 $v $round', d['ms_per_step'])"
  done
done
