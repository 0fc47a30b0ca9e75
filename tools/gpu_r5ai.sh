#!/bin/bash
# round 5: the epilogue tables loaded in the first slab, stored in the second -- tests, bench A/B
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r5ai; mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "dx3 or fused or teacher_forced or lanes or dxb or codec or config3 or flips" > $O/t.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|Error" $O/t.log | tail -4; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
for v in new prev; do
  if [ $v = new ]; then L=""; else L=tools/ab_lib/prev/libidfcodec.so; fi
  IDF_LIB_PATH=$L timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-residual --no-cpu-baseline > $O/bench_$v.$rep.json 2> $O/bench_$v.$rep.err || exit 1
  python3 -c "import json; d=json.load(open('$O/bench_$v.$rep.json')); print('$v', d['value'], d['serial'], d['roofline']['frac'])"
done
done
for v in new prev; do
  if [ $v = new ]; then L=""; else L=tools/ab_lib/prev/libidfcodec.so; fi
  for c in resflow-cond-imagenet64 resflows_smallpatch_split; do
    IDF_LIB_PATH=$L timeout -k 10 300 python -u tools/bench_residual.py --config $c > $O/res_${v}_$c.json 2> $O/res_${v}_$c.err || exit 1
    python3 -c "import json; d=json.load(open('$O/res_${v}_$c.json')); r=d.get('roofline', {}); print('$v $c', d.get('value'), r.get('frac'))"
  done
done
