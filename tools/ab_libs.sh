#!/bin/bash
# A/B of library builds on one box: bench (1 engine, K3 event = solo kernel
# time) alternating between libwebp_amd_<variant>.so builds.
# Usage: bash tools/ab_libs.sh <tag> <variant>... ("main" = libwebp_amd.so)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=$1; shift; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
for round in 1 2; do
  for v in "$@"; do
    lib=$R/libwebp_amd/libwebp_amd_$v.so; [ "$v" = main ] && lib=$R/libwebp_amd/libwebp_amd.so
    WEBP_AMD_LIB=$lib timeout -k 10 120 python3 bench.py --no-cpu --no-host-input --engines 1 \
      --steps 6 --warmup 1 > $O/${v}_$round.json 2> $O/${v}_$round.err || exit 1
  done
done
echo done > $O/done
