#!/bin/bash
# Lossless line with / without the double-buffered upload, then the default
# lossy line as the driver runs it.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/$1; mkdir -p $O; cd $R
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --no-cpu --lossless > $O/lpf_$i.json 2> $O/lpf_$i.err || exit 1
  timeout -k 10 300 python3 bench.py --no-cpu --lossless --no-prefetch > $O/lnp_$i.json 2> $O/lnp_$i.err || exit 1
done
timeout -k 10 400 python3 bench.py > $O/bench0.json 2> $O/bench0.err || exit 1
echo done > $O/done
