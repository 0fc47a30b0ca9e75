#!/bin/bash
# round 5: encode lanes (IDF_ENC_LANES=2) and four decode streams per block (IDF_DECODE_WPB=4)
# re-measured on the round-5 kernels -- bench A/B
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r5ar; mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
for rep in 1 2; do
for v in base enc2 wpb4; do
  case $v in base) E="";; enc2) E="IDF_ENC_LANES=2";; wpb4) E="IDF_DECODE_WPB=4";; esac
  env $E timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-residual --no-cpu-baseline > $O/bench_$v.$rep.json 2> $O/bench_$v.$rep.err || exit 1
  python3 -c "import json; d=json.load(open('$O/bench_$v.$rep.json')); print('$v', d['value'], d['serial'], d['round_trip_exact_steps'])"
done
done
