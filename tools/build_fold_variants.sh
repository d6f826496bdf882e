#!/bin/bash
# Measurement only: libgloo_amd.so with the k-source chain folds issuing
# every source's loads first (FOLD_PRELOAD=1) under
# tools/fold_variants/<name>/, for A/B against the default (source by
# source).  Load one with GLOO_AMD_LIB=<that .so>.  Built here.
set -e
cd "$(dirname "$0")/.."
make -C gloo_amd -j8 >/dev/null
HIPFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Iinclude -Igloo_amd/include"
OBJS=$(ls gloo_amd/build/*.o | grep -v reduce.hip.o)
build() {  # name defines...
  local name=$1; shift
  mkdir -p tools/fold_variants/$name
  hipcc $HIPFLAGS -mllvm -amdgpu-kernarg-preload-count=16 "$@" -c gloo_amd/csrc/reduce.hip -o tools/fold_variants/$name/reduce.o
  hipcc --offload-arch=gfx950 -shared $OBJS tools/fold_variants/$name/reduce.o -o tools/fold_variants/$name/libgloo_amd.so
  rm tools/fold_variants/$name/reduce.o
}
build preload -DFOLD_PRELOAD=1
ls -la tools/fold_variants/*/
