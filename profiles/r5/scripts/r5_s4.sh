#!/bin/bash
# Round-5 session 4: the intra-4 || chroma fork (K3): parity suite, stage
# split, bench line.
set -o pipefail
O=gpurun_out/${1:-r5s4}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_token_fallbacks.py tests/test_multipass.py tests/test_autofilter.py \
  tests/test_shards.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python -u bench.py --no-cpu > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]);print(d['value'],d.get('hbm_resident_mps'),d['ms_per_step'],d['roofline']['k_encode_solo_ms'],d['stage_ms'])"
WEBP_AMD_LIB=libwebp_amd/libwebp_amd_prof.so timeout -k 10 120 python -u tools/k3_stages.py 1920 1080 256 4 > $O/k3_stages_256.log 2>&1 || exit 1
grep -v amdgpu.ids $O/k3_stages_256.log
