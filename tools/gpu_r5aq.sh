#!/bin/bash
# round 5: do rANS decode kernels slow the L0 convs beside them? (pipelined bench kernel trace)
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r5aq; mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
R=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr -o run --output-format csv -- python3 -u bench.py --steps 6 --warmup 2 --no-residual --no-cpu-baseline > $O/bench.log 2>&1 || exit $?
f=$(ls $O/tr/*kernel_trace.csv $O/tr/*/*kernel_trace.csv 2>/dev/null | head -1)
python3 tools/analysis/overlap.py "$f" > $O/overlap.txt || exit 1
rm -rf $O/tr
cat $O/overlap.txt
