#!/bin/bash
# Decode streams per block (IDF_DECODE_WPB 4 / 2 / 1): the chain alone (rans_bench_0) and the
# codec bench, same box.
set -u -o pipefail
cd "$(dirname "$0")/.."
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/wpb; mkdir -p $O
for w in 4 2 1; do echo "== WPB $w"; IDF_DECODE_WPB=$w timeout -k 10 60 ./tools/native/rans_bench_0 2>&1 | grep -v amdgpu.ids || exit 1; done | tee $O/chain.txt
for r in 1 2; do
  for w in 4 2; do
    IDF_DECODE_WPB=$w timeout -k 10 200 python3 -u bench.py --no-residual --no-cpu-baseline --steps 10 --warmup 2 > $O/b_${w}_$r.json 2>$O/err.log || { tail -5 $O/err.log; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b_${w}_$r.json')); print('WPB $w', d['value'], 'ms', d['ms_per_step'], 'serial', d.get('serial'), 'exact', d['round_trip_exact'])"
  done
done | tee $O/ab.txt
