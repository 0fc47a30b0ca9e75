#!/bin/bash
# Timing-only ablations of the wq kernel (tools/wq_ablate.sh variants) at L0 c=144/496, L1 c=504.
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/wq_ablate
mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
for r in 1 2; do
  for n in 0; do
    echo "== wq_$n"
    IDF_LIB_PATH=tools/wq_lib/wq_$n/libidfcodec.so IDF_WQ=1 KB_ONLY=wx3 KB_LEVELS=0,1 KB_LAYERS=3,11 \
      timeout -k 10 120 python3 -u tools/kbench.py 2>&1 | grep -v amdgpu.ids || exit $?
  done
  echo "== wx3 (IDF_WQ=0)"
  IDF_WQ=0 KB_ONLY=wx3 KB_LEVELS=0,1 KB_LAYERS=3,11 timeout -k 10 120 python3 -u tools/kbench.py 2>&1 | grep -v amdgpu.ids || exit $?
done > $O/ablate.log 2>&1
cat $O/ablate.log
