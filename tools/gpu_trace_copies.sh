#!/bin/bash
# kernel + memory-copy trace of a short bench run; summarise where the copyBuffer blits come from
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/trace_copies
mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace -d $O/raw -o run --output-format csv -- python3 -u bench.py --no-residual --no-cpu-baseline --steps 2 --warmup 1 > $O/bench.log 2>&1 || exit $?
python3 tools/trace_copies.py $O/raw > $O/summary.txt 2>&1
cat $O/summary.txt
rm -rf $O/raw
