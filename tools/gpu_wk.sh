#!/bin/bash
# wk conv GPU step: parity tests of the K=32 split-f16 Winograd kernel, then the per-layer
# kernel timing of wx3 vs wk at the imagenet64 shapes (tools/kbench.py).
set -u -o pipefail
cd "$(dirname "$0")/.."
O=${O:-gpurun_out/wk}
mkdir -p "$O"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_wk.py > "$O/wk_tests.log" 2>&1; rc=$?
tail -25 "$O/wk_tests.log"
[ $rc -eq 0 ] || exit $rc
KB_ONLY=wx3,wk KB_LAYERS=0,3,6,9,11 KB_REPS=10 timeout -k 10 240 python -u tools/kbench.py > "$O/kbench.log" 2>&1 || exit $?
cat "$O/kbench.log"
