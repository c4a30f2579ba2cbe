#!/bin/bash
# Build A/B variants of libmep_hip.so that differ only in csrc/attn.hip compile-time switches:
#   VARIANTS="name=-DFLAG=1 -DX=2;name2=..." bash scripts/build_variants.sh
# -> variants/<name>/libmep_hip.so (the other objects from the main build).  Run here (CPU); the
# .so files travel to the GPU box with the tree (git-ignored).
set -e
cd "$(dirname "$0")/.."
C=multimodal-emotion-processing_amd/csrc
make -s -C $C -j8
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -mllvm -disable-promote-alloca-to-lds -I../../include -fno-slp-vectorize"
IFS=';' read -ra VS <<< "$VARIANTS"
pids=()
for v in "${VS[@]}"; do
  name=${v%%=*}; flags=${v#*=}
  mkdir -p variants/$name
  ( cd $C && /opt/rocm/bin/hipcc $FLAGS $flags -c attn.hip -o ../../variants/$name/attn.o && \
    /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ../../variants/$name/libmep_hip.so \
      $(ls build/*.o | grep -v attn.o) ../../variants/$name/attn.o && echo "built $name ($flags)" ) &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
