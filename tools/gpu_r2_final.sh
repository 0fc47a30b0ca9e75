#!/bin/bash
# Round-end evidence at HEAD: the full GPU suite, smoke, the default bench line, a rocprofv3
# kernel-trace summary of the bench, the HBM traffic passes the bench's roofline.traffic reads
# (tools/pmc_bench.sh) and the wx3 SQ counter passes (tools/pmc_x3.sh).  Every GPU step has
# its own time limit; the first failure ends the script.
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/final
mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1; rc=$?
tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bench", d["value"], d["ms_per_step"], d["encode_ms"], d["decode_ms"], d["round_trip_exact"], d["roofline"]["frac"])'
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 -u bench.py --no-residual --no-cpu-baseline > $O/prof.log 2>&1 || exit $?
cp $O/prof/run_kernel_stats.csv $O/kernel_stats.csv
head -6 $O/kernel_stats.csv | cut -c1-150
./tools/pmc_bench.sh || exit $?
OUT=$O/pmc_x3 ./tools/pmc_x3.sh || exit $?
python tools/pmc_summary.py $O/pmc_x3 > $O/pmc_x3/summary.txt 2>&1 || true
echo final done
