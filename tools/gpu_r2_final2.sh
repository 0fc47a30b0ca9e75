#!/bin/bash
# Round-end evidence at the last commit: GPU suite, smoke, bench line, rocprofv3 kernel stats.
set -u -o pipefail
cd "$(dirname "$0")/.."
O=${O:-gpurun_out/final2}
mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1; rc=$?
tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bench", d["value"], d["ms_per_step"], d["encode_ms"], d["decode_ms"], d["round_trip_exact"], d["roofline"]["frac"], d["roofline"]["avg_launch_ms"])'
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 -u bench.py --no-residual --no-cpu-baseline > $O/prof.log 2>&1 || exit $?
f=$(ls $O/prof/*kernel_stats.csv $O/prof/*/*kernel_stats.csv 2>/dev/null | head -1); cp "$f" $O/kernel_stats.csv
head -6 $O/kernel_stats.csv | cut -c1-150
echo final2 done
