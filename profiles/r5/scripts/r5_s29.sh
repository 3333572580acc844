#!/bin/bash
# Round-5 session 29: snapshot interval A/B (8 / 16 / 32 MBs) on the batch
# K3 and config 4; traces of both with snapshots.
set -o pipefail
O=gpurun_out/${1:-r5s29}
mkdir -p $O
bash tools/k3_ab.sh ${1:-r5s29}ab main snap8 snap32 || exit 1
for v in main snap8 snap32; do
  lib=$(pwd)/libwebp_amd/libwebp_amd_$v.so; [ $v = main ] && lib=$(pwd)/libwebp_amd/libwebp_amd.so
  WEBP_AMD_LIB=$lib timeout -k 10 200 python3 bench.py --batch 1 --width 4096 --height 4096 --quality 90 --method 6 \
    --steps 2 --warmup 1 --no-host-input --no-cpu --engines 1 > $O/cfg4_$v.json 2> $O/cfg4_$v.err || exit 1
  python3 -c "import json;d=json.loads(open('$O/cfg4_$v.json').read().strip().splitlines()[-1]);print('cfg4 $v', d['ms_per_step'])"
done
bash tools/gpu_session.sh ${1:-r5s29} trace trace4 || exit 1
for t in 256 cfg4; do python3 -c "import json;d=json.load(open('$O/k3_trace_$t.json'));print('$t', d['k_encode_ms'], d['share_of_worker_cycles'])"; done
