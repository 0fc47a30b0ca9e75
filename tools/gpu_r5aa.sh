#!/bin/bash
# round 5: per-layer dx3 durations in the serial bench (kernel trace), kept as a summary
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r5aa; mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
R=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr -o run --output-format csv -- python3 -u bench.py --steps 3 --warmup 1 --pipeline 0 --no-residual --no-cpu-baseline > $O/bench.log 2>&1 || exit $?
f=$(ls $O/tr/*kernel_trace.csv $O/tr/*/*kernel_trace.csv 2>/dev/null | head -1)
python3 tools/analysis/layer_times.py "$f" > $O/layer_times.txt || exit 1
python3 tools/analysis/trace_util.py "$f" 2 > $O/util.txt 2>&1
rm -rf $O/tr
cat $O/layer_times.txt
