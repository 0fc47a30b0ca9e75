#!/bin/bash
set -u -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_production_parity.py > gpurun_out/r2b_parity.log 2>&1; rc=$?
tail -3 gpurun_out/r2b_parity.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
OUT=gpurun_out/pmc_x3_head ./tools/pmc_x3.sh || exit $?
./tools/pmc_bench.sh || exit $?
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_head -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-residual --steps 3 --warmup 1 > gpurun_out/prof_head.log 2>&1; rc=$?
tail -c 600 gpurun_out/prof_head.log; exit $rc
