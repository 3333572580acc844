#!/bin/bash
# Timeline of the default bench line: kernels + memory copies with the frames
# uploaded from host memory, and kernels alone with the frames in HBM.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/$1; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/host -o run \
  -- python3 $R/bench.py --no-cpu --steps ${STEPS:-18} --warmup 1 --no-other-input > $O/host.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/hbm -o run \
  -- python3 $R/bench.py --no-cpu --no-host-input --steps ${STEPS:-18} --warmup 1 --no-other-input > $O/hbm.log 2>&1 || exit 1
echo done > $O/done
