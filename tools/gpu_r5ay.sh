#!/bin/bash
# round 5: back-to-back (serial) encode / decode timeline from a kernel trace
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r5ay; mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
R=$(pwd); cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr -o run --output-format csv -- python3 -u bench.py --pipeline 0 --steps 4 --warmup 1 --no-residual --no-cpu-baseline > $O/bench.log 2>&1 || exit 1
f=$(ls $O/tr/*kernel_trace.csv $O/tr/*/*kernel_trace.csv 2>/dev/null | head -1); cp "$f" $O/kernel_trace.csv; rm -rf $O/tr
for k in 2 3 4; do python3 tools/analysis/decode_timeline.py $O/kernel_trace.csv $k; done > $O/serial_timeline.txt; rm -f $O/kernel_trace.csv; cat $O/serial_timeline.txt
tail -1 $O/bench.log | cut -c1-300
