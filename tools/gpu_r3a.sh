#!/bin/bash
# Round 3: GPU tests touched by the dist / host-ABI / log_prob changes, then the N=2 rehearsal.
set -u -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_production_parity.py tests/test_gpu_dist_staged.py tests/test_gpu_codec.py \
  tests/test_gpu_lanes.py tests/test_gpu_residual.py > gpurun_out/r3a_tests.log 2>&1 || {
  tail -c 4000 gpurun_out/r3a_tests.log; exit 1; }
tail -n 3 gpurun_out/r3a_tests.log
bash tools/gpu_rehearse2.sh
