#!/bin/bash
# Pipelined bench under decode-lane settings (same box): IDF_LANES x IDF_LANE_STAGGER.
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/pipe_lanes; mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
for r in 1 2; do
  for v in "2 flows0" "1 flows0" "2 top" "2 none" "4 flows0"; do
    set -- $v
    IDF_LANES=$1 IDF_LANE_STAGGER=$2 timeout -k 10 200 python3 -u bench.py --no-residual --no-cpu-baseline --steps 10 --warmup 2 2>/dev/null > $O/b.json || exit 1
    python3 -c "import json; d=json.load(open('$O/b.json')); print('lanes=$1 stagger=$2', d['value'], 'ms', d['ms_per_step'], 'enc', d['encode_ms'], 'dec', d['decode_ms'], 'exact', d['round_trip_exact'])"
  done
done | tee $O/ab.txt
