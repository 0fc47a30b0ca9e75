#!/bin/bash
# Same-box A/B of the dx3 prefix width (IDF_DX3_CMAX "L0,L1": widest 16-padded layer input on
# dx3 per level; unset = every layer, IDF_DX3=0 = none), after a per-layer wx3/dx3 sweep.
# The IDF_DX3_CMAX hook was taken out after this A/B (engine._dx3_cmax: every layer on dx3;
# results in profiles/r04/dx3_prefix/).
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/cmax; mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
KB_ONLY=wx3,dx3 KB_LEVELS=0,1 KB_LAYERS=0,1,2,3,4,5,6,7,8,9,10,11 \
  timeout -k 10 150 python3 -u tools/kbench.py > $O/kbench.log 2>&1 || { tail -5 $O/kbench.log; exit 1; }
for r in 1 2; do
  for v in ${CMAX_VARIANTS:-all none 232,152 144,108}; do
    case $v in
      all) env_="" ;;
      none) env_="IDF_DX3=0" ;;
      *) env_="IDF_DX3_CMAX=$v" ;;
    esac
    env $env_ timeout -k 10 200 python3 -u bench.py --no-residual --no-cpu-baseline --steps 10 --warmup 2 2>$O/err_${v}_$r.log > $O/b_${v}_$r.json || { tail -5 $O/err_${v}_$r.log; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b_${v}_$r.json')); print('cmax=$v', d['value'], 'ms', d['ms_per_step'], 'enc', d['encode_ms'], 'dec', d['decode_ms'], 'exact', d['round_trip_exact'], 'frac', d['roofline']['frac'], 'serial', d.get('serial'))"
  done
done | tee $O/ab.txt
