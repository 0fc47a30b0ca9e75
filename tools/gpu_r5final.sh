#!/bin/bash
# round 5 closing measurements at the final sources: smoke, the GPU suite, the default bench line,
# its rocprofv3 kernel stats, and the PMC traffic passes (profiles/r05/final, profiles/r05/pmc_bench)
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r5final; mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
tail -1 $O/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=15 > $O/gpu_suite.log 2>&1
rc=$?; echo "suite rc=$rc"; grep -E "passed|failed" $O/gpu_suite.log | tail -2; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['serial'], d['roofline'], d['cpu_baseline'], d['round_trip_exact_steps'])"
O=$O/prof timeout -k 10 700 bash tools/gpu_prof.sh > /dev/null 2>&1 || exit 1
head -8 $O/prof/kernel_stats.csv | cut -d, -f1-4
timeout -k 10 900 bash tools/pmc_bench.sh || exit 1
