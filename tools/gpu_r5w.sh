#!/bin/bash
# round 5: lane 1 started after lane 0's first k top-level couplings too (IDF_LANE_LEAD), serial
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r5w; mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
for rep in 1 2; do
  for k in 0 2 4 8; do
    IDF_LANE_LEAD=$k timeout -k 10 200 python -u bench.py --pipeline 0 --steps 6 --warmup 2 --no-residual --no-cpu-baseline > $O/lead$k.$rep.json 2> $O/lead$k.$rep.err || exit 1
    python3 -c "import json; d=json.load(open('$O/lead$k.$rep.json')); print('lead $k', d['value'], d['encode_ms'], d['decode_ms'], d['round_trip_exact_steps'])"
  done
done
