#!/bin/bash
# Headline-only kernel profile: bench.py without the residual configs and the CPU baseline.
set -u -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/prof_head
export PYTHONDONTWRITEBYTECODE=1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_head -o run -- \
  python3 bench.py --steps 5 --warmup 1 --no-residual --no-cpu-baseline > gpurun_out/prof_head/bench.log 2>&1
rc=$?
tail -c 1500 gpurun_out/prof_head/bench.log
find gpurun_out/prof_head -name "*kernel_stats.csv" | head -3
exit $rc
