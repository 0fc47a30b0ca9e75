#!/bin/bash
# Decode-lane stagger with the two-streams-per-block decode: back-to-back bench, same box.
set -u -o pipefail
cd "$(dirname "$0")/.."
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/stagger; mkdir -p $O
for r in 1 2; do
  for v in ${STAG_VARIANTS:-flows0 top flows none}; do
    IDF_LANE_STAGGER=$v timeout -k 10 200 python3 -u bench.py --no-residual --no-cpu-baseline --pipeline ${PIPE:-0} --steps 10 --warmup 2 > $O/b_${v}_$r.json 2>$O/err.log || { tail -5 $O/err.log; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b_${v}_$r.json')); print('$v', d['value'], 'enc', d['encode_ms'], 'dec', d['decode_ms'], 'exact', d['round_trip_exact'])"
  done
done | tee $O/ab.txt
