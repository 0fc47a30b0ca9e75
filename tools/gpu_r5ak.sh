#!/bin/bash
# round 5: config 4's kernel split (rocprofv3 kernel stats of tools/bench_residual.py)
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r5ak; mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
R=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 -u tools/bench_residual.py --config resflows_smallpatch_split --steps 2 > $O/res.json 2> $O/res.err || exit $?
f=$(ls $O/prof/*kernel_stats.csv $O/prof/*/*kernel_stats.csv 2>/dev/null | head -1); cp "$f" $O/kernel_stats.csv
t=$(ls $O/prof/*kernel_trace.csv $O/prof/*/*kernel_trace.csv 2>/dev/null | head -1)
python3 tools/analysis/layer_times.py "$t" > $O/layer_times.txt
rm -rf $O/prof
head -16 $O/kernel_stats.csv | cut -d, -f1-5
