#!/bin/bash
# round 5: split stores as 16-B octets (C % 8 == 0) -- tests, bench A/B, kbench
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r5ax; mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "dx3 or fused or teacher_forced or codec or lanes or flow or config45" > $O/t.log 2>&1
rc=$?; echo "dx3 tests rc=$rc"; grep -E "passed|failed|Error" $O/t.log | tail -4; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
for v in new prev; do
  if [ $v = new ]; then L=""; else L=tools/ab_lib/prev/libidfcodec.so; fi
  IDF_LIB_PATH=$L timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-residual --no-cpu-baseline > $O/bench_$v.$rep.json 2> $O/bench_$v.$rep.err || exit 1
  python3 -c "import json; d=json.load(open('$O/bench_$v.$rep.json')); print('$v', d['value'], d['serial'], d['roofline']['frac'], d['round_trip_exact_steps'])"
done
done
for v in new prev; do
  if [ $v = new ]; then L=""; else L=tools/ab_lib/prev/libidfcodec.so; fi
  IDF_LIB_PATH=$L KB_B=128 KB_ONLY=dx3 KB_LEVELS=0,1,2 KB_LAYERS=0,6,11 timeout -k 10 200 python -u tools/kbench.py > $O/kb_$v.log 2>&1 || exit 1
  grep -v amdgpu $O/kb_$v.log | sed "s/^/$v /"
done
