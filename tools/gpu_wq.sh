#!/bin/bash
# wq kernel: parity tests (wq + wx3 routing), then a same-process layer benchmark A/B
# (IDF_WQ=0 runs the old wx3 kernel) at the imagenet64 L0/L1 shapes.
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/wq
mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_wq.py > $O/tests.log 2>&1; rc=$?
tail -5 $O/tests.log
[ $rc -ne 0 ] && exit $rc
for v in 0 1 0 1; do
  echo "== IDF_WQ=$v"
  IDF_WQ=$v KB_ONLY=wx3 KB_LEVELS=0,1 KB_LAYERS=0,3,6,9,11 timeout -k 10 120 python3 -u tools/kbench.py || exit $?
done > $O/kbench.log 2>&1
cat $O/kbench.log
