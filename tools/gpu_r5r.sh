#!/bin/bash
# round 5: dxb (bf16 direct conv) layer timings and ablations (kbench, B=1024 at 32x32 and
# 16x16, the config-3 batch) vs the old bf16 kernel, same box
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r5r; mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
KB_B=1024 KB_ONLY=dxb,bf16 KB_LEVELS=0,1,2 KB_LAYERS=0,3,6,9,11 timeout -k 10 200 python -u tools/kbench.py > $O/base.log 2>&1 || exit 1
cat $O/base.log
for v in abl_nohalo abl_now abl_nodma abl_nobar abl_nomfma; do
  IDF_LIB_PATH=tools/ab_lib/$v/libidfcodec.so KB_B=1024 KB_ONLY=dxb KB_LEVELS=0,1,2 KB_LAYERS=0,6,11 timeout -k 10 200 python -u tools/kbench.py > $O/$v.log 2>&1 || exit 1
  echo "== $v"; cat $O/$v.log
done
