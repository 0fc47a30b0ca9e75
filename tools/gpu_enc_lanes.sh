#!/bin/bash
# Encode lanes: exactness tests, then a same-box bench A/B of IDF_ENC_LANES=1 vs 2.
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/enc_lanes
mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_lanes.py > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log
[ $rc -ne 0 ] && exit $rc
for r in 1 2 3; do
  for e in 1 2; do
    IDF_ENC_LANES=$e timeout -k 10 180 python3 -u bench.py --no-residual --no-cpu-baseline --steps 10 --warmup 2 2>/dev/null > $O/b_${e}_$r.json || exit $?
    python3 -c "import json; d=json.load(open('$O/b_${e}_$r.json')); print('enc_lanes $e', d['value'], 'enc', d['encode_ms'], 'dec', d['decode_ms'], 'exact', d['round_trip_exact'], 'frac', d['roofline']['frac'])"
  done
done | tee $O/summary.txt
