#!/bin/bash
# PC sampling of K3 (rocprofv3 host-trap sampling, beta): which instructions
# of k_encode<4> the waves sit on, for one 256 x 1080p batch (two launches).
set -o pipefail
O=gpurun_out/${1:-r5pcs}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
timeout -s KILL 60 rocprofv3 -L > $R/$O/list.txt 2>&1 || true
grep -i -A12 "pc sampl\|PC_SAMPLING\|host_trap\|stochastic" $R/$O/list.txt | head -40
timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method ${2:-host_trap} \
  --pc-sampling-unit ${3:-time} --pc-sampling-interval ${4:-1} --kernel-include-regex k_encode \
  -d $R/$O/pcs -o pcs --output-format csv -- python3 $R/tools/k3_stages.py 1920 1080 256 4 \
  > $R/$O/pcs.log 2>&1 || { echo "pc sampling failed"; tail -20 $R/$O/pcs.log; exit 1; }
find $R/$O/pcs -name "*.csv" | head; 
