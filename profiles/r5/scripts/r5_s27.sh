#!/bin/bash
# Round-5 session 27: K3X statistics snapshots (replay starts at the last
# 16-MB boundary before a counter's halving point): parity, then config 4
# A/B against the build without them.
set -o pipefail
O=gpurun_out/${1:-r5s27}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_multipass.py tests/test_token_fallbacks.py \
  tests/test_alpha.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for round in 1 2; do
  for v in main nosnap; do
    lib=$(pwd)/libwebp_amd/libwebp_amd_$v.so; [ $v = main ] && lib=$(pwd)/libwebp_amd/libwebp_amd.so
    WEBP_AMD_LIB=$lib timeout -k 10 200 python3 bench.py --batch 1 --width 4096 --height 4096 --quality 90 --method 6 \
      --steps 2 --warmup 1 --no-host-input --no-cpu --engines 1 > $O/cfg4_${v}_$round.json 2> $O/cfg4_${v}_$round.err || exit 1
    python3 -c "import json;d=json.loads(open('$O/cfg4_${v}_$round.json').read().strip().splitlines()[-1]);print('cfg4 $v $round', d['ms_per_step'])"
  done
done
