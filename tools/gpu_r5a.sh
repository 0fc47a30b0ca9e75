#!/bin/bash
# round 5: the packed / split-K dx3 -- kernel parity, then the imagenet64 8x8 level's blocks
# teacher-forced, then the codec's conv modes (dx3 at every level, dx3w16 legacy files).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_dx3.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/r5a_dx3_tests.log 2>&1
rc=$?; echo "dx3 tests rc=$rc"; tail -15 gpurun_out/r5a_dx3_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_production_parity.py -x -v --timeout 200 \
  --timeout-method thread -k "teacher_forced and dx3" -s > gpurun_out/r5a_parity.log 2>&1
rc=$?; echo "parity rc=$rc"; grep -E "level|passed|failed|Error" gpurun_out/r5a_parity.log | tail -12
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_codec.py -x -v --timeout 200 --timeout-method thread \
  -k "conv_modes or range_guard_clean" > gpurun_out/r5a_codec.log 2>&1
rc=$?; echo "codec rc=$rc"; tail -5 gpurun_out/r5a_codec.log
exit $rc
