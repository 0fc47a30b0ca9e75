#!/bin/bash
# Builds libidfcodec.so variants with conv3_dx3.hip compiled under extra -D flags into
# tools/ab_lib/<name>/ (timing A/Bs on the GPU box through IDF_LIB_PATH).
# Usage: tools/dx3_build_knobs.sh name1 "-DIDF_DX3_DB=5" name2 "-DIDF_DX3_SB=0" ...
set -eu
cd "$(dirname "$0")/.."
PKG=finalproject-losslessimagecompression_amd
make -s -C $PKG
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -I$PKG/csrc -Wno-unused-result"
OBJS=$(ls $PKG/build/*.o | grep -v conv3_dx3.o)
names=()
while [ $# -ge 2 ]; do
  n=$1; d=tools/ab_lib/$n; mkdir -p $d; names+=($n)
  /opt/rocm/bin/hipcc $FLAGS $2 -c $PKG/csrc/conv3_dx3.hip -o $d/conv3_dx3.o &
  shift 2
done
wait
for n in "${names[@]}"; do
  d=tools/ab_lib/$n
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OBJS $d/conv3_dx3.o -o $d/libidfcodec.so
done
