#!/bin/bash
# host-input bench under the runtime's copy-engine settings (which engine
# carries the H2D upload: blit kernels need CUs that K3 holds, SDMA does not)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=${1:-h2d}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
for v in default 2 1; do
  if [ $v = default ]; then E=""; else E="GPU_BLIT_ENGINE_TYPE=$v"; fi
  env $E timeout -k 10 200 python3 bench.py --no-cpu --steps 4 --warmup 1 > $O/bench_$v.json 2> $O/bench_$v.err
  rc=$?; echo "blit $v rc=$rc" >> $O/steps.log; [ $rc = 0 ] || exit $rc
done
