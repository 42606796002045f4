#!/bin/bash
# Build libotmatch.so with extra compile flags into reporter_amd/lib/variants/<name>/ (A/B of compile-time knobs):
#   bash scripts/build_variant.sh cap8 -DOTM_CAND_LANE_CAP=8
set -e
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/reporter_amd/lib/variants/$NAME
mkdir -p $OUT/obj
cd $ROOT/reporter_amd/csrc
FLAGS="-O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -I../../include -I. $*"
/opt/rocm/bin/hipcc $FLAGS --offload-arch=gfx950 -c kernels.hip -o $OUT/obj/kernels.o
# engine.cpp shares kernels.h's constants (buffer sizes): built with the same flags
/opt/rocm/bin/hipcc $FLAGS -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ -x c++ -c engine.cpp -o $OUT/obj/engine.o
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $OUT/libotmatch.so \
  $(ls ../lib/obj/*.o | grep -v -e kernels.o -e engine.o) $OUT/obj/kernels.o $OUT/obj/engine.o -lpthread
echo $OUT/libotmatch.so
