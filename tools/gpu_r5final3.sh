#!/bin/bash
# round 5 closing measurements at the final sources: PMC traffic passes first (installed into
# profiles/r05/pmc_bench of this box's copy so the bench line reports traffic), then smoke, the
# GPU suite, the default bench line and its rocprofv3 kernel stats (all under gpurun_out/r5final3)
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r5final3; mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 900 bash tools/pmc_bench.sh || exit 1
cp gpurun_out/pmc_bench/fetch.csv gpurun_out/pmc_bench/write.csv gpurun_out/pmc_bench/source_hash.txt profiles/r05/pmc_bench/ || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
tail -1 $O/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=15 > $O/gpu_suite.log 2>&1
rc=$?; echo "suite rc=$rc"; grep -E "passed|failed" $O/gpu_suite.log | tail -2; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
python3 -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print(d['value'], d['serial'], r['frac'], r['traffic'], r.get('traffic_over_algorithmic'), d['round_trip_exact_steps']); print({k: (v.get('value'), v.get('roofline', {}).get('frac')) for k, v in (d.get('residual_configs') or {}).items()})"
O=$O/prof timeout -k 10 700 bash tools/gpu_prof.sh > /dev/null 2>&1 || exit 1
head -6 $O/prof/kernel_stats.csv | cut -d, -f1-4
