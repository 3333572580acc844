#!/bin/bash
# A/B library build: libwebp_amd/libwebp_amd_<name>.so with vp8_k3.hip
# compiled under extra -D options (the other objects from the main build),
# then the lane-mask ISA check. Usage: bash tools/build_variant.sh <name> -DX=1 ...
set -e
R=$(cd "$(dirname "$0")/.." && pwd); N=$1; shift
cd $R/libwebp_amd/csrc
/opt/rocm/bin/hipcc -O3 -fPIC -fvisibility=hidden -std=c++17 --offload-arch=gfx950 -Wno-unused-result \
  -I$R/include -I$R/libwebp_amd/csrc "$@" -c hip/vp8_k3.hip -o $R/build/obj/vp8_k3_$N.o
cd $R/build/obj
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -Wl,-Bsymbolic -o $R/libwebp_amd/libwebp_amd_$N.so \
  webp_api.o picture_enc.o vp8_host.o gpu_batch.o picture_tools.o vp8l_host.o vp8l_batch.o host_cpus.o \
  h2d_sdma.o vp8_kernels.o vp8_k3_$N.o vp8_emit.o vp8_sharp.o vp8l_kernels.o vp8_autofilter.o \
  -lpthread -lm -L/opt/rocm/lib -lhsa-runtime64
python3 $R/tools/isa_lane0_check.py $R/libwebp_amd/libwebp_amd_$N.so
