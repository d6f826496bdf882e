#!/bin/bash
# Measurement only: libgloo_amd.so variants whose interpreter kernels use
# another block size / unroll (reduce.hip GLOO_AMD_INTERP_*), each under
# tools/interp_variants/<name>/ (LD_LIBRARY_PATH=<that dir> overrides the
# RUNPATH of tools/latency).  Built here, on the CPU.
set -e
cd "$(dirname "$0")/.."
make -C gloo_amd -j8 >/dev/null
HIPFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Iinclude -Igloo_amd/include"
OBJS=$(ls gloo_amd/build/*.o | grep -v reduce.hip.o)
build() {  # name defines...
  local name=$1; shift
  mkdir -p tools/interp_variants/$name
  hipcc $HIPFLAGS "$@" -c gloo_amd/csrc/reduce.hip -o tools/interp_variants/$name/reduce.o
  hipcc --offload-arch=gfx950 -shared $OBJS tools/interp_variants/$name/reduce.o -o tools/interp_variants/$name/libgloo_amd.so
  rm tools/interp_variants/$name/reduce.o
}
build b512_c8_f4 -DGLOO_AMD_INTERP_COPY_UNROLL=8 -DGLOO_AMD_INTERP_FOLD_UNROLL=4 &
build b1024_c4_f2 -DGLOO_AMD_INTERP_BLOCK=1024 &
build b1024_c8_f4 -DGLOO_AMD_INTERP_BLOCK=1024 -DGLOO_AMD_INTERP_COPY_UNROLL=8 -DGLOO_AMD_INTERP_FOLD_UNROLL=4 &
build b256_c8_f4 -DGLOO_AMD_INTERP_BLOCK=256 -DGLOO_AMD_INTERP_COPY_UNROLL=8 -DGLOO_AMD_INTERP_FOLD_UNROLL=4 &
wait
ls -la tools/interp_variants/*/
