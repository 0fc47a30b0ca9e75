#!/bin/bash
# Same-box A/B: pipelined steps (step k's decode beside step k+1's encode) vs back to back.
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/pipe; mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
for r in 1 2; do
  for p in 1 0; do
    timeout -k 10 200 python3 -u bench.py --no-residual --no-cpu-baseline --steps 10 --warmup 2 --pipeline $p 2>$O/err_${p}_$r.log > $O/b_${p}_$r.json || { tail -5 $O/err_${p}_$r.log; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b_${p}_$r.json')); print('pipeline=$p', d['value'], 'ms', d['ms_per_step'], 'enc', d['encode_ms'], 'dec', d['decode_ms'], 'exact', d['round_trip_exact'], 'serial', d.get('serial'))"
  done
done | tee $O/ab.txt
