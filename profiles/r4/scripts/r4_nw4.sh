#!/bin/bash
# 4-worker K3 with tokens copied in K3: the config-3 shard loop (3 then 4
# workers, diagnostic build), then the GPU suite, bench, the host-input copy
# trace and rocprof kernel stats on the product build. Stops at the first
# failing step.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=${1:-r4i}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
for v in 5 4; do
  WEBP_AMD_LIB=$R/libwebp_amd/libwebp_amd_diag.so WEBP_AMD_K3=$v timeout -k 10 100 \
    python3 -u tools/shard_probe.py > $O/shard_k3_$v.log 2>&1
  rc=$?; echo "shard k3=$v rc=$rc" >> $O/steps.log; [ $rc = 0 ] || exit $rc
done
bash tools/gpu_session.sh $T tests bench copytrace prof
