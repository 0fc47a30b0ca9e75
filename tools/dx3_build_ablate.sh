#!/bin/bash
# Builds timing-only variants of libidfcodec.so with conv3_dx3.hip compiled under
# -DIDF_DX3_ABLATE=N into tools/ab_lib/dx3_N/ (run here, on the CPU; the GPU box only loads
# them through IDF_LIB_PATH).  Usage: tools/dx3_build_ablate.sh 0 7 8 16 96 15
set -eu
cd "$(dirname "$0")/.."
PKG=finalproject-losslessimagecompression_amd
make -s -C $PKG
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -I$PKG/csrc -Wno-unused-result"
OBJS=$(ls $PKG/build/*.o | grep -v conv3_dx3.o)
for n in "$@"; do
  d=tools/ab_lib/dx3_$n; mkdir -p $d
  /opt/rocm/bin/hipcc $FLAGS -DIDF_DX3_ABLATE=$n -c $PKG/csrc/conv3_dx3.hip -o $d/conv3_dx3.o &
done
wait
for n in "$@"; do
  d=tools/ab_lib/dx3_$n
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OBJS $d/conv3_dx3.o -o $d/libidfcodec.so
done
