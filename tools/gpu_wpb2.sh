#!/bin/bash
# Two streams per decode block as the default: the decode suites, then a same-box bench A/B.
set -u -o pipefail
cd "$(dirname "$0")/.."
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/wpb2; mkdir -p $O
[ -n "${SKIP_TESTS:-}" ] || timeout -k 10 800 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_rans.py \
  tests/test_gpu_codec.py tests/test_gpu_lanes.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
[ -n "${SKIP_TESTS:-}" ] || tail -1 $O/tests.log
for r in 1 2; do
  for w in ${WPB_VARIANTS:-4 2}; do
    IDF_DECODE_WPB=$w timeout -k 10 200 python3 -u bench.py --no-residual --no-cpu-baseline --steps 10 --warmup 2 > $O/b_${w}_$r.json 2>$O/err.log || { tail -5 $O/err.log; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b_${w}_$r.json')); print('WPB $w', d['value'], 'ms', d['ms_per_step'], 'enc', d['encode_ms'], 'dec', d['decode_ms'], 'serial', d.get('serial'), 'exact', d['round_trip_exact'], 'rans', d.get('rans', {}).get('decode', {}).get('ns_per_symbol'))"
  done
done | tee $O/ab.txt
