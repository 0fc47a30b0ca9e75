#!/bin/bash
# round 2, first GPU pass: new parity tests, the full -m gpu suite, bench (with residual extras)
set -u -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_production_parity.py > gpurun_out/r2a_parity.log 2>&1; rc=$?
tail -25 gpurun_out/r2a_parity.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests --deselect tests/test_gpu_production_parity.py > gpurun_out/r2a_gpu.log 2>&1; rc=$?
tail -8 gpurun_out/r2a_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -u bench.py > gpurun_out/r2a_bench.log 2>&1; rc=$?
tail -c 3000 gpurun_out/r2a_bench.log
exit $rc
