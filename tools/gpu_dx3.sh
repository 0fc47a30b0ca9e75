#!/bin/bash
# dx3 probe: parity tests of the split-f16 direct conv, then wx3 vs dx3 per layer (kbench).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_dx3.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/dx3_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -25 gpurun_out/dx3_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
KB_ONLY=${KB_ONLY:-wx3,dx3} KB_LEVELS=${KB_LEVELS:-0,1} KB_LAYERS=${KB_LAYERS:-0,3,6,9,11} \
  timeout -k 10 300 python -u tools/kbench.py > gpurun_out/dx3_kbench.log 2>&1
rc=$?; echo "kbench rc=$rc"; cat gpurun_out/dx3_kbench.log
exit $rc
