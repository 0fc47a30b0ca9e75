#!/bin/bash
# rocprofv3 kernel stats of the headline bench (default steps, no residual configs, no CPU
# baseline) into $O/kernel_stats.csv, and the bench line it printed.
set -u -o pipefail
cd "$(dirname "$0")/.."
O=${O:-gpurun_out/prof}
mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
R=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 -u bench.py --no-residual --no-cpu-baseline ${BENCH_ARGS:-} > $O/prof.log 2>&1 || exit $?
f=$(ls $O/prof/*kernel_stats.csv $O/prof/*/*kernel_stats.csv 2>/dev/null | head -1); cp "$f" $O/kernel_stats.csv
rm -rf $O/prof
head -14 $O/kernel_stats.csv | cut -d, -f1-5
tail -1 $O/prof.log | cut -c1-400
