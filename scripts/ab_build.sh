#!/bin/bash
# Build the variants of an A/B on the CPU host, before the GPU call:
#   VARIANTS="base=;occ2=-DMEP_WG_OCC_BF=2" bash scripts/ab_build.sh
# -> variants/<name>/lib.so (git-ignored, shipped to the box by gpurun), used by scripts/ab.sh.
cd "$(dirname "$0")/.."
IFS=';' read -ra VS <<< "$VARIANTS"
for v in "${VS[@]}"; do
  name=${v%%=*}; flags=${v#*=}
  rm -rf variants/$name
  make -s -C multimodal-emotion-processing_amd/csrc -j8 EXTRA="$flags" BUILD=$PWD/variants/$name/obj \
    OUT=$PWD/variants/$name/lib.so > /tmp/ab_build_$name.log 2>&1 || { echo "build $name failed"; tail -5 /tmp/ab_build_$name.log; exit 1; }
  rm -rf variants/$name/obj
  echo "built variants/$name/lib.so"
done
