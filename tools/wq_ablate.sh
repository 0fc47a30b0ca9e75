#!/bin/bash
# Build timing-only ablation variants of libidfcodec.so (conv3_wq.hip with -DIDF_WQ_ABLATE=N)
# into tools/wq_lib/wq_N/ for same-box A/Bs (IDF_LIB_PATH); the other objects are the tree's.
set -eu
cd "$(dirname "$0")/.."
P=finalproject-losslessimagecompression_amd
for n in "$@"; do
  d=tools/wq_lib/wq_$n; mkdir -p $d
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize \
    -I$P/csrc -DIDF_WQ_ABLATE=$n -c $P/csrc/conv3_wq.hip -o $d/conv3_wq.o
  objs=$(ls $P/build/*.o | grep -v conv3_wq.o)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs $d/conv3_wq.o -o $d/libidfcodec.so
  rm $d/conv3_wq.o
done
