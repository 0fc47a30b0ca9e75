#!/bin/bash
# Unequal decode lanes (IDF_LANE_SPLIT: lane 0's share) under the "top" stagger, same box.
set -u -o pipefail
cd "$(dirname "$0")/.."
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/split; mkdir -p $O
for r in 1 2; do
  for p in 1 0; do
    for v in 0.5 0.4375 0.5625; do
      IDF_LANE_SPLIT=$v timeout -k 10 200 python3 -u bench.py --no-residual --no-cpu-baseline --pipeline $p --steps 10 --warmup 2 > $O/b_${p}_${v}_$r.json 2>$O/err.log || { tail -5 $O/err.log; exit 1; }
      python3 -c "import json; d=json.load(open('$O/b_${p}_${v}_$r.json')); print('pipe $p split $v', d['value'], 'enc', d['encode_ms'], 'dec', d['decode_ms'], 'exact', d['round_trip_exact'])"
    done
  done
done | tee $O/ab.txt
