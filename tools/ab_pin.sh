#!/bin/bash
# A/B of host-thread placement and K3 solo time (one GPU box session)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${1:-ab}; mkdir -p $O; cd $R
B="python3 $R/bench.py --no-cpu --no-host-input --steps 10 --warmup 2"
timeout -k 10 200 $B > $O/pin.json 2> $O/pin.err || exit 1
WEBP_AMD_NO_PIN=1 timeout -k 10 200 $B > $O/nopin.json 2> $O/nopin.err || exit 1
timeout -k 10 200 $B > $O/pin2.json 2> $O/pin2.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run \
  -- python3 $R/bench.py --no-cpu --no-host-input --steps 3 --warmup 1 --engines 1 > $O/prof.log 2>&1 || exit 1
echo done > $O/done
