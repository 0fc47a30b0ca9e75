#!/bin/bash
# round 5: the default bench line (10 timed steps) at the final sources, and its kernel stats
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r5final4; mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
python3 -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print(d['value'], d['steps'], d['serial'], r['frac'], r['traffic'], r.get('traffic_over_algorithmic'), d['round_trip_exact_steps'], d['cpu_baseline']['value'], d['cpu_baseline'].get('gpu_over_cpu_encode')); print({k: (v.get('value'), v.get('roofline', {}).get('frac')) for k, v in (d.get('residual_configs') or {}).items()})"
O=$O/prof timeout -k 10 700 bash tools/gpu_prof.sh > /dev/null 2>&1 || exit 1
head -4 $O/prof/kernel_stats.csv | cut -d, -f1-4
