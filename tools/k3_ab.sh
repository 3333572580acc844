#!/bin/bash
# K3 timing A/B of library builds (timing-only variants allowed: no output
# check): k_encode of one 256 x 1080p q75 m4 launch (the second of two, one
# engine, HIP events) per build, two rounds alternating.
# Usage: bash tools/k3_ab.sh <tag> <variant>... ("main" = libwebp_amd.so)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=$1; shift; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
for round in 1 2; do
  for v in "$@"; do
    lib=$R/libwebp_amd/libwebp_amd_$v.so; [ "$v" = main ] && lib=$R/libwebp_amd/libwebp_amd.so
    WEBP_AMD_LIB=$lib timeout -k 10 120 python3 tools/k3_stages.py 1920 1080 256 4 \
      > $O/${v}_$round.log 2>&1 || { rc=$?; echo "$v failed rc=$rc"; tail -5 $O/${v}_$round.log; exit 1; }
    echo "$v $round: $(grep -o 'k_encode [0-9.]* ms' $O/${v}_$round.log)"
  done
done
