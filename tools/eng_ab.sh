#!/bin/bash
# Encoder instances per GPU on the default (host-input) line: 4 / 5 / 6
# instances, three timed steps each, two rounds.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/$1; mkdir -p $O; cd $R
for i in 1 2; do
  for e in ${ENGS:-4 5 6}; do
    timeout -k 10 300 python3 bench.py --no-cpu --steps $((3 * e)) --warmup 2 --engines $e \
      > $O/eng${e}_$i.json 2> $O/eng${e}_$i.err || exit 1
  done
done
echo done > $O/done
