#!/bin/bash
# Build A/B variants of libmep_hip.so that differ in compile-time switches of some csrc files:
#   VARIANTS="name=-DFLAG=1 -DX=2;name2=..." [VFILES="attn.hip block.hip"] bash scripts/build_variants.sh
# -> variants/<name>/libmep_hip.so (VFILES recompiled with the flags, the other objects from the
# main build).  Run here (CPU); the .so files travel to the GPU box with the tree (git-ignored).
set -e
cd "$(dirname "$0")/.."
C=multimodal-emotion-processing_amd/csrc
make -s -C $C -j8
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -mllvm -disable-promote-alloca-to-lds -I../../include"
VFILES=${VFILES:-attn.hip}
IFS=';' read -ra VS <<< "$VARIANTS"
pids=()
for v in "${VS[@]}"; do
  name=${v%%=*}; flags=${v#*=}
  mkdir -p variants/$name
  (
    cd $C
    objs=""
    for f in $VFILES; do
      o=../../variants/$name/${f%.hip}.o
      extra=""; [ "$f" = attn.hip ] && extra="-fno-slp-vectorize"
      /opt/rocm/bin/hipcc $FLAGS $extra $flags -c $f -o $o
      objs="$objs $o"
    done
    keep=""
    for o in build/*.o; do b=$(basename $o .o); case " $VFILES " in *" $b.hip "*) ;; *) keep="$keep $o";; esac; done
    /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ../../variants/$name/libmep_hip.so $keep $objs && echo "built $name ($flags)"
  ) &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
