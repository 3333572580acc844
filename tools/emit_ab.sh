#!/bin/bash
# K4 A/B builds: libwebp_amd_<name>.so with vp8_emit.hip compiled with other
# EMIT_IMG (tokens k_emit_img looks back) / MAP_G (segments per k_emit_maps
# wave). Build here: bash tools/emit_ab.sh build; on the box:
# bash tools/emit_ab.sh run <tag> <name>...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}; cd $R
declare -A FL=([i512g8]="-DEMIT_IMG=512 -DMAP_G=8" [i512g16]="-DEMIT_IMG=512 -DMAP_G=16"
               [i1024g16]="-DEMIT_IMG=1024 -DMAP_G=16" [i256g16]="-DEMIT_IMG=256 -DMAP_G=16")
if [ "$1" = build ]; then
  O=$R/build/obj; C=$R/libwebp_amd/csrc
  for v in "${!FL[@]}"; do
    /opt/rocm/bin/hipcc -O3 -fPIC -fvisibility=hidden -std=c++17 --offload-arch=gfx950 -Wno-unused-result \
      -I$R/include -I$C ${FL[$v]} -c $C/hip/vp8_emit.hip -o $O/vp8_emit_$v.o || exit 1
    objs=$(ls $O/*.o | grep -v -e vp8_emit -e _ab_ -e _trace -e _diag -e _stamps -e _prof)
    /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -Wl,-Bsymbolic -o $R/libwebp_amd/libwebp_amd_$v.so \
      $objs $O/vp8_emit_$v.o -lpthread -lm -L/opt/rocm/lib -lhsa-runtime64 || exit 1
  done
  exit 0
fi
T=$2; shift 2; D=$R/gpurun_out/$T; mkdir -p $D
for v in "$@"; do
  lib=$R/libwebp_amd/libwebp_amd_$v.so; [ "$v" = main ] && lib=$R/libwebp_amd/libwebp_amd.so
  WEBP_AMD_LIB=$lib timeout -k 10 120 python -u -m pytest tests/test_emit_gpu.py -m gpu -x -q --timeout 100 \
    --timeout-method thread > $D/tests_$v.log 2>&1 || exit 1
  (cd /tmp && TMPDIR=/tmp WEBP_AMD_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $D/st_$v -o run -- python3 $R/bench.py --no-cpu --no-host-input --steps 3 --warmup 1 --engines 1 \
    > $D/bench_$v.json 2> $D/bench_$v.err) || exit 1
done
echo done > $D/done
