#!/bin/bash
# round 5: block timelines of L0 layers 0 / 5 / 11 at one lane's batch (128 images)
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r5ab; mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
for l in 0 5 11; do
  IDF_LIB_PATH=tools/ab_lib/tl/libidfcodec.so KB_B=128 KB_LEVELS=0 KB_LAYERS=$l timeout -k 10 120 python -u tools/dx3_timeline.py > $O/tl_l0_$l.log 2>&1 || exit 1
  echo "== L0 layer $l"; grep -v amdgpu.ids $O/tl_l0_$l.log
done
