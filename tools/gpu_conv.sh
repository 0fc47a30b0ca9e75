#!/bin/bash
# conv GPU step: the Winograd / wx3 parity tests and the production-parity x3 blocks, then the
# ablation harness timing (tools/native/wino_ablate_0, wino_stamps).
set -u -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_wx3.py tests/test_gpu_wino.py tests/test_gpu_production_parity.py -k "not config3_full" > gpurun_out/conv_tests.log 2>&1; rc=$?
tail -5 gpurun_out/conv_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 60 ./tools/native/wino_ablate_0 x3 > gpurun_out/conv_time.log 2>&1 || exit $?
timeout -k 10 60 ./tools/native/wino_stamps x3 >> gpurun_out/conv_time.log 2>&1 || exit $?
cat gpurun_out/conv_time.log
