#!/bin/bash
# kernel + memory-copy trace of a short bench run (which kernels and copies land inside a step)
set -u -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace -d gpurun_out/trace -o run --output-format csv -- python -u bench.py --no-residual --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/trace.log 2>&1 || exit $?
tail -c 1500 gpurun_out/trace.log
find gpurun_out/trace -name "*.csv" | xargs ls -la
