#!/bin/bash
# Same-box timing of the dx3 knob variants (tools/dx3_build_knobs.sh) at the L0/L1 wide layers.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
for r in 1 2; do
  for n in ${VARIANTS}; do
    echo "== $n"
    IDF_LIB_PATH=$PWD/tools/ab_lib/$n/libidfcodec.so KB_ONLY=dx3 KB_LEVELS=0,1 \
      KB_LAYERS=${KB_LAYERS:-3,11} timeout -k 10 120 python -u tools/kbench.py 2>&1 | grep -v amdgpu.ids
    rc=$?; [ $rc -eq 0 ] || exit $rc
  done
done
