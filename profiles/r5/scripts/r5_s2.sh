#!/bin/bash
# Round-5 session 2: the whole GPU suite on the pooled host threads, the
# 4-worker trace build's hang records (check build), one default bench line.
set -o pipefail
O=gpurun_out/r5s2
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ \
  > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]);print(d['value'],d.get('hbm_resident_mps'),d['ms_per_step'],d['stage_ms'])"
WEBP_AMD_LIB=libwebp_amd/libwebp_amd_tracecheck.so timeout -k 10 300 \
  python -u tools/k3_trace.py 1920 1080 256 4 75 $O/k3_trace_nw4.json > $O/tracecheck.log 2>&1 || { echo "tracecheck failed"; tail -20 $O/tracecheck.log; exit 1; }
grep -E "K3_CHECK|K3_HANG" $O/tracecheck.log | head -30
grep k_encode_ms $O/k3_trace_nw4.json
