#!/bin/bash
# Round-3 evidence, part B: the default bench line (CPU pool + residual configs) and a rocprofv3
# kernel-stats profile of the headline bench.
set -u -o pipefail
cd "$(dirname "$0")/.."
O=${O:-gpurun_out/r3final}
mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 700 python -u bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["cpu_baseline"]; print("bench", d["value"], d["ms_per_step"], d["encode_ms"], d["decode_ms"], d["round_trip_exact"], d["roofline"]["frac"], d["roofline"]["avg_launch_ms"], "cpu", c.get("value"), c.get("cores"), c.get("split"), c.get("effective_cpus"))'
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 -u bench.py --no-residual --no-cpu-baseline > $O/prof.log 2>&1 || exit $?
f=$(ls $O/prof/*kernel_stats.csv $O/prof/*/*kernel_stats.csv 2>/dev/null | head -1); cp "$f" $O/kernel_stats.csv
head -6 $O/kernel_stats.csv | cut -c1-150
tail -1 $O/prof.log | cut -c1-300
