#!/bin/bash
# round 5: head running sums loaded before the epilogue's stores -- tests, bench + kbench A/B
# against the previous library (tools/ab_lib/prev)
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r5y; mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "dx3 or fused or teacher_forced or lanes or dxb" > $O/t.log 2>&1
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
  IDF_LIB_PATH=$L KB_ONLY=dx3 KB_LEVELS=0,1,2 KB_LAYERS=0,6,11 timeout -k 10 200 python -u tools/kbench.py > $O/kb_$v.log 2>&1 || exit 1
  grep -v amdgpu $O/kb_$v.log | sed "s/^/$v /"
done
