#!/bin/bash
# Encode lanes (IDF_ENC_LANES 1 vs 2) with the round-4 decode settings, same box.
set -u -o pipefail
cd "$(dirname "$0")/.."
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/enc_lanes_r4; mkdir -p $O
for r in 1 2; do
  for p in 1 0; do
    for v in 1 2; do
      IDF_ENC_LANES=$v timeout -k 10 200 python3 -u bench.py --no-residual --no-cpu-baseline --pipeline $p --steps 10 --warmup 2 > $O/b_${p}_${v}_$r.json 2>$O/err.log || { tail -5 $O/err.log; exit 1; }
      python3 -c "import json; d=json.load(open('$O/b_${p}_${v}_$r.json')); print('pipe $p enc_lanes $v', d['value'], 'enc', d['encode_ms'], 'dec', d['decode_ms'], 'exact', d['round_trip_exact'])"
    done
  done
done | tee $O/ab.txt
