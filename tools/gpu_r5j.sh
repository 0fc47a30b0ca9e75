#!/bin/bash
# round 5: DMA spread knobs of the branch-free DMA issue (L0/L1 kbench, alternating builds)
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r5j; mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
for rep in 1 2; do
  for v in base dmas2 dmas3 dma0_12; do
    IDF_LIB_PATH=tools/ab_lib/$v/libidfcodec.so KB_ONLY=dx3 KB_LEVELS=0,1 KB_LAYERS=0,3,6,9,11 KB_REPS=20 \
      timeout -k 10 300 python -u tools/kbench.py > $O/kb_${v}_$rep.log 2>&1 || exit 1
    echo "$v $rep $(grep 'sampled total' $O/kb_${v}_$rep.log) L0c496 $(grep 'c= 496' $O/kb_${v}_$rep.log | awk '{print $6}') L1c504 $(grep 'c= 504' $O/kb_${v}_$rep.log | awk '{print $6}')"
  done
done
