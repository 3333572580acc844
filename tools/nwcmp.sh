#!/bin/bash
# k_encode time for 1/2/3/4 MB workers per frame (WEBP_AMD_K3 variants)
set -e -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out/nw
for V in ${@:-3 5 4}; do
  WEBP_AMD_K3=$V timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu > $R/gpurun_out/nw/b$V.log 2>&1
done
echo done
