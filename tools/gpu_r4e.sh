#!/bin/bash
# Round 4: parity after the 8x8 epilogue remap / dx3 prologue reorder / concurrent encode,
# then per-layer timing, the 8x8 SQ counters, the pipelined-bench A/B, dx3 phase stamps and the
# bench decode timeline.
set -u -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 500 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_dx3.py tests/test_gpu_wx3.py tests/test_gpu_wino.py "tests/test_gpu_production_parity.py::test_imagenet64_x3_blocks_teacher_forced" "tests/test_gpu_lanes.py::test_encode_beside_decode_exact" > gpurun_out/r4e_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r4e_tests.log; [ $rc -eq 0 ] || exit $rc
KB_ONLY=wx3,dx3 KB_LEVELS=0,1 KB_LAYERS=0,3,6,9,11 timeout -k 10 300 python -u tools/kbench.py > gpurun_out/r4e_kbench.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r4e_kbench.log
bash tools/gpu_pipe_ab.sh || exit $?
IDF_LIB_PATH=$PWD/tools/ab_lib/stamps/libidfcodec.so timeout -k 10 120 python3 tools/dx3_stamps.py > gpurun_out/stamps_phase.txt 2>&1 || exit $?
tail -8 gpurun_out/stamps_phase.txt
OUT=gpurun_out/pmc_x3_r4 bash tools/pmc_x3.sh > /dev/null || exit $?
python3 tools/pmc_summary.py gpurun_out/pmc_x3_r4 conv3_wino > gpurun_out/pmc_x3_r4/summary.txt 2>&1
bash tools/gpu_trace_r4.sh
