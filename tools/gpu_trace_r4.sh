#!/bin/bash
# kernel trace of a short bench run, then the decode timeline of its steps
set -u -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace -d gpurun_out/trace -o run --output-format csv -- python3 -u bench.py --no-residual --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/trace.log 2>&1 || exit $?
f=$(find gpurun_out/trace -name "*kernel_trace.csv" | head -1)
for k in 1 2 3; do python3 tools/analysis/decode_timeline.py $f $k; done | tee gpurun_out/decode_timeline.txt
