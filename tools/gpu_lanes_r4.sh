#!/bin/bash
# Decode lanes 2 vs 3 with the two-stream decode blocks and the "top" stagger, same box.
set -u -o pipefail
cd "$(dirname "$0")/.."
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/lanes_r4; mkdir -p $O
for r in 1 2; do
  for p in 1 0; do
    for n in 2 3; do
      IDF_LANES=$n timeout -k 10 200 python3 -u bench.py --no-residual --no-cpu-baseline --pipeline $p --steps 10 --warmup 2 > $O/b_${p}_${n}_$r.json 2>$O/err.log || { tail -5 $O/err.log; exit 1; }
      python3 -c "import json; d=json.load(open('$O/b_${p}_${n}_$r.json')); print('pipe $p lanes $n', d['value'], 'enc', d['encode_ms'], 'dec', d['decode_ms'], 'exact', d['round_trip_exact'])"
    done
  done
done | tee $O/ab.txt
