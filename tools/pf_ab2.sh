#!/bin/bash
# Instances per GPU with the double-buffered upload: 5 / 6 with it, 5 without.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/$1; mkdir -p $O; cd $R
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --no-cpu --engines 5 --steps 15 > $O/pf5_$i.json 2> $O/pf5_$i.err || exit 1
  timeout -k 10 300 python3 bench.py --no-cpu --engines 5 --steps 15 --no-prefetch > $O/np5_$i.json 2> $O/np5_$i.err || exit 1
  timeout -k 10 300 python3 bench.py --no-cpu --engines 6 --steps 18 > $O/pf6_$i.json 2> $O/pf6_$i.err || exit 1
  timeout -k 10 300 python3 bench.py --no-cpu --engines 4 --steps 12 > $O/pf4_$i.json 2> $O/pf4_$i.err || exit 1
done
echo done > $O/done
