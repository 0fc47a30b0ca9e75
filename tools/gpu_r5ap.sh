#!/bin/bash
# round 5: decode lane stagger "flowstop" (every lane's top-level rANS decode at t = 0, lane i's
# top-level couplings after lane i-1's) vs the default "top" -- bench A/B (serial numbers too)
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r5ap; mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
for rep in 1 2; do
for v in flowstop top; do
  IDF_LANE_STAGGER=$v timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-residual --no-cpu-baseline > $O/bench_$v.$rep.json 2> $O/bench_$v.$rep.err || exit 1
  python3 -c "import json; d=json.load(open('$O/bench_$v.$rep.json')); print('$v', d['value'], d['serial'], d['round_trip_exact_steps'])"
done
done
