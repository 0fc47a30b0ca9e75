#!/bin/bash
# round 5: fused heads of up to 32 outputs -- tests, bench A/B against the 16-output cap
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r5x; mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -s -k "dx3 or fused or teacher_forced or config45 or lanes or codec or flips or forward_vs or bf16 or config3" > $O/t.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "flips|passed|failed|Error" $O/t.log | tail -6; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for h in 32 16; do
    IDF_DX3_HEAD_MAX=$h timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-residual --no-cpu-baseline > $O/bench_h$h.$rep.json 2> $O/bench_h$h.$rep.err || exit 1
    python3 -c "import json; d=json.load(open('$O/bench_h$h.$rep.json')); print('hmax $h', d['value'], d['serial'], d['roofline']['frac'])"
  done
done
for c in resflow-cond-imagenet64 resflows_smallpatch_split; do
  timeout -k 10 300 python -u tools/bench_residual.py --config $c > $O/res_$c.json 2> $O/res_$c.err || exit 1
  python3 -c "import json; d=json.load(open('$O/res_$c.json')); r=d.get('roofline', {}); print('$c', d.get('value'), r.get('frac'))"
done
