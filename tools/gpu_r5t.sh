#!/bin/bash
# round 5: where the bench's device-to-device copies come from (pipelined default run, trace)
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r5t; mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
R=$(pwd); cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr -o run --output-format csv -- python3 -u bench.py --steps 4 --warmup 1 --no-residual --no-cpu-baseline > $O/bench.log 2>&1 || exit 1
f=$(ls $O/tr/*kernel_trace.csv $O/tr/*/*kernel_trace.csv 2>/dev/null | head -1); cp "$f" $O/kernel_trace.csv; rm -rf $O/tr
echo ok
