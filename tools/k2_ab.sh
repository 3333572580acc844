#!/bin/bash
# K2 timing A/B builds (vp8_kernels.hip with extra -D flags): build here with
# bash tools/k2_ab.sh build; on the box: bash tools/k2_ab.sh run <tag> <name>...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}; cd $R
declare -A FL=([noatom]="-DK2_NO_ATOMIC")
if [ "$1" = build ]; then
  O=$R/build/obj; C=$R/libwebp_amd/csrc
  for v in "${!FL[@]}"; do
    /opt/rocm/bin/hipcc -O3 -fPIC -fvisibility=hidden -std=c++17 --offload-arch=gfx950 -Wno-unused-result \
      -I$R/include -I$C ${FL[$v]} -c $C/hip/vp8_kernels.hip -o $O/vp8_kernels_$v.o || exit 1
    objs=$(ls $O/*.o | grep -v -e vp8_kernels -e _ab_ -e _trace -e _diag -e _stamps -e _prof -e vp8_emit_)
    /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -Wl,-Bsymbolic -o $R/libwebp_amd/libwebp_amd_$v.so \
      $objs $O/vp8_kernels_$v.o -lpthread -lm -L/opt/rocm/lib -lhsa-runtime64 || exit 1
  done
  exit 0
fi
T=$2; shift 2; D=$R/gpurun_out/$T; mkdir -p $D
for v in "$@"; do
  lib=$R/libwebp_amd/libwebp_amd_$v.so; [ "$v" = main ] && lib=$R/libwebp_amd/libwebp_amd.so
  (cd /tmp && TMPDIR=/tmp WEBP_AMD_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $D/st_$v -o run -- python3 $R/bench.py --no-cpu --no-host-input --steps 2 --warmup 1 --engines 1 \
    > $D/bench_$v.json 2> $D/bench_$v.err) || exit 1
done
echo done > $D/done
