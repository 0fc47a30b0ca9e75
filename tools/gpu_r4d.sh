#!/bin/bash
# Round 4: wx3 parity after the 8x8 epilogue lane remap, its SQ counters (bank conflicts), then
# the bench kernel trace and decode timeline.
set -u -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_wx3.py tests/test_gpu_wino.py "tests/test_gpu_production_parity.py::test_imagenet64_x3_blocks_teacher_forced" > gpurun_out/wx3_tests.log 2>&1; rc=$?
tail -3 gpurun_out/wx3_tests.log; [ $rc -eq 0 ] || exit $rc
OUT=gpurun_out/pmc_x3_r4 bash tools/pmc_x3.sh || exit $?
python3 tools/pmc_summary.py gpurun_out/pmc_x3_r4 conv3_wino > gpurun_out/pmc_x3_r4/summary.txt 2>&1
bash tools/gpu_trace_r4.sh
