#!/bin/bash
# Round-5 session 7: the K3 fork (intra-16 + chroma on the fourth wave beside
# intra-4), per-wave intra-4 records, barrier fast path, prefetched MB source,
# branch-free edge loads: parity, bench, stages; timing A/B of the prefetch
# and of the token statistics atomics; config 4 / one 1080p frame; the trace
# build (four workers) on the 256 x 1080p batch.
set -o pipefail
bash tools/r5_s4.sh r5s7 || exit 1
bash tools/k3_ab.sh r5s7ab main nopf nostat || exit 1
O=gpurun_out/r5s7
timeout -k 10 300 python3 bench.py --batch 1 --width 4096 --height 4096 --quality 90 --method 6 \
  --steps 2 --warmup 1 --no-host-input --no-cpu --engines 1 > $O/bench_cfg4.json 2> $O/bench_cfg4.err || { echo cfg4 failed; tail -5 $O/bench_cfg4.err; exit 1; }
timeout -k 10 300 python3 bench.py --batch 1 --steps 10 --warmup 2 --no-host-input --no-cpu \
  --engines 1 > $O/bench_1080p_single.json 2> $O/bench_1080p_single.err || { echo single failed; exit 1; }
python3 -c "
import json
for f in ('bench_cfg4','bench_1080p_single'):
    d=json.loads(open('$O/'+f+'.json').read().strip().splitlines()[-1]); print(f, d['value'], d['ms_per_step'], d['roofline']['k_encode_solo_ms'])"
WEBP_AMD_LIB=libwebp_amd/libwebp_amd_tracecheck.so timeout -k 10 200 \
  python -u tools/k3_trace.py 1920 1080 256 4 75 $O/k3_trace_nw4.json > $O/tracecheck.log 2>&1 || { echo "tracecheck failed"; tail -20 $O/tracecheck.log; exit 1; }
grep -E "K3_CHECK|K3_HANG" $O/tracecheck.log | head; grep k_encode_ms $O/k3_trace_nw4.json
