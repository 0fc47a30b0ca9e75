#!/bin/bash
# round 2: full GPU suite, smoke, then the bench with a rocprofv3 kernel-trace summary.
set -u -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r2d_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/r2d_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r2d_smoke.log 2>&1 || exit $?
tail -2 gpurun_out/r2d_smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/r2d_bench.log 2>&1 || exit $?
tail -c 2500 gpurun_out/r2d_bench.log
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 60 ./tools/native/wino_stamps x3 > gpurun_out/r2d_conv_time.log 2>&1 && cat gpurun_out/r2d_conv_time.log && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r2d_prof -o run --output-format csv -- python -u bench.py --no-residual --no-cpu-baseline > gpurun_out/r2d_prof.log 2>&1 || exit $?
find gpurun_out/r2d_prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/r2d_kernel_stats.csv
head -12 gpurun_out/r2d_kernel_stats.csv
