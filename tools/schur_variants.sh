#!/usr/bin/env bash
# Compile variants of the HIP library with different k_schur tuning macros into tools/lib_<name>.so (CPU, in this
# container); tools/schur_probe.py times k_schur for each on the GPU.  usage: tools/schur_variants.sh name:"-DX=1 ..." ...
set -e
cd "$(dirname "$0")/.."
mkdir -p build/variants
for spec in "$@"; do
  name="${spec%%:*}"; defs="${spec#*:}"
  (
    for src in ba_kernels passes tracks; do
      obj=build/obj/$src.hip.o
      if [ $src = ba_kernels ]; then
        obj=build/variants/${name}_$src.o
        /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -munsafe-fp-atomics $defs -c -o $obj \
          instantsfm_amd/csrc/$src.hip
      fi
    done
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ${OUTDIR:-tools}/lib_$name.so build/variants/${name}_ba_kernels.o \
      build/obj/passes.hip.o build/obj/tracks.hip.o
    echo "built ${OUTDIR:-tools}/lib_$name.so ($defs)"
  ) &
done
wait
