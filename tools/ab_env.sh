#!/bin/bash
# A/B of environment settings on one box: bench lines alternating between
# settings given as NAME=ENV strings ("base" = none), e.g.
#   bash tools/ab_env.sh <tag> base k3v6:WEBP_AMD_K3=6 e3:ENGINES=3
# (ENGINES=n is passed as --engines n)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=$1; shift; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
for round in 1 2; do
  for spec in "$@"; do
    name=${spec%%:*}; envs=""; extra=""
    [ "$spec" != "$name" ] && envs=${spec#*:}
    for kv in ${envs//,/ }; do
      case $kv in ENGINES=*) extra="--engines ${kv#ENGINES=}";; *) export_kv="$export_kv $kv";; esac
    done
    env $export_kv timeout -k 10 150 python3 bench.py --no-cpu --no-host-input $extra --steps 6 \
      --warmup 1 > $O/${name}_$round.json 2> $O/${name}_$round.err || exit 1
    export_kv=""
  done
done
echo done > $O/done
