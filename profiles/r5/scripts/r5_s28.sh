#!/bin/bash
# Round-5 session 28: statistics snapshots in the batch K3 too: parity
# (whole GPU suite), batch K3 A/B against the build without snapshots,
# config 4 and single-frame lines.
set -o pipefail
O=gpurun_out/${1:-r5s28}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests \
  > $O/tests.log 2>&1 || { echo "tests failed rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/k3_ab.sh ${1:-r5s28}ab main nosnap || exit 1
timeout -k 10 300 python3 bench.py --batch 1 --width 4096 --height 4096 --quality 90 --method 6 \
  --steps 3 --warmup 1 --no-host-input --no-cpu --engines 1 > $O/bench_cfg4.json 2> $O/bench_cfg4.err || exit 1
for v in main nosnap; do
  lib=$(pwd)/libwebp_amd/libwebp_amd_$v.so; [ $v = main ] && lib=$(pwd)/libwebp_amd/libwebp_amd.so
  WEBP_AMD_LIB=$lib timeout -k 10 300 python3 bench.py --batch 1 --steps 10 --warmup 2 --no-host-input --no-cpu \
    --engines 1 > $O/bench_1080p_single_$v.json 2> $O/bench_1080p_single_$v.err || exit 1
done
for f in bench_cfg4 bench_1080p_single_main bench_1080p_single_nosnap; do python3 -c "import json;d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]);print('$f', d['value'], d['ms_per_step'])"; done
