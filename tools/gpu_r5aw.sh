#!/bin/bash
# round 5: split K at images of <= 16 pixels (config 4's 4x4 and 2x2 levels: a few dozen tiles,
# latency-bound launches) -- dx3 / config 4 parity on the variant, config 4 bench A/B
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r5aw; mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
IDF_LIB_PATH=tools/ab_lib/sp16/libidfcodec.so timeout -k 10 400 python -u -m pytest tests/test_gpu_dx3.py tests/test_gpu_production_parity.py -x -q --timeout 300 --timeout-method thread -s -k "(dx3 or config45) and not supported_geometry" > $O/t.log 2>&1
rc=$?; echo "tests (sp16) rc=$rc"; grep -E "smallpatch|passed|failed|Error" $O/t.log | tail -8; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
for v in sp16 base; do
  if [ $v = base ]; then L=""; else L=tools/ab_lib/$v/libidfcodec.so; fi
  c=resflows_smallpatch_split
  IDF_LIB_PATH=$L timeout -k 10 300 python -u tools/bench_residual.py --config $c > $O/res_${v}_$rep.json 2> $O/res_${v}_$rep.err || exit 1
  python3 -c "import json; d=json.load(open('$O/res_${v}_$rep.json')); r=d.get('roofline', {}); print('$v', d.get('value'), d.get('encode_ms'), d.get('decode_ms'), r.get('frac'), d.get('round_trip_exact'))"
done
done
