#!/bin/bash
# Round-5 session 24: the K3X row fold's replay with 16 chunks per step:
# parity subset, config 4 and single-frame lines, config 4 trace.
set -o pipefail
O=gpurun_out/${1:-r5s24}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_token_fallbacks.py tests/test_multipass.py tests/test_autofilter.py \
  tests/test_shards.py tests/test_concurrency.py tests/test_alpha.py > $O/tests.log 2>&1 || { echo "tests failed rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python3 bench.py --batch 1 --width 4096 --height 4096 --quality 90 --method 6 \
  --steps 3 --warmup 1 --no-host-input --no-cpu --engines 1 > $O/bench_cfg4.json 2> $O/bench_cfg4.err || exit 1
timeout -k 10 300 python3 bench.py --batch 1 --steps 10 --warmup 2 --no-host-input --no-cpu \
  --engines 1 > $O/bench_1080p_single.json 2> $O/bench_1080p_single.err || exit 1
for f in bench_cfg4 bench_1080p_single; do python3 -c "import json;d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]);print('$f', d['value'], d['ms_per_step'])"; done
bash tools/gpu_session.sh ${1:-r5s24} trace4 || exit 1
python3 -c "import json;d=json.load(open('$O/k3_trace_cfg4.json'));print(d['k_encode_ms'], d['cycles_per_mb'])"
bash tools/k3_ab.sh ${1:-r5s24}ab main prev || exit 1
