#!/bin/bash
# round 5: only the leading waves (0-3) issue the split kernel's DMA pieces (IDF_DX3_DMAW=4) --
# dx3 tests on the variant, kbench and bench A/B
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r5au; mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
IDF_LIB_PATH=tools/ab_lib/dw4/libidfcodec.so timeout -k 10 300 python -u -m pytest tests/test_gpu_dx3.py -x -q --timeout 250 --timeout-method thread > $O/t.log 2>&1
rc=$?; echo "dx3 tests (dw4) rc=$rc"; grep -E "passed|failed|Error" $O/t.log | tail -3; [ $rc -ne 0 ] && exit $rc
for v in dw4 base; do
  if [ $v = base ]; then L=""; else L=tools/ab_lib/$v/libidfcodec.so; fi
  IDF_LIB_PATH=$L KB_B=128 KB_ONLY=dx3 KB_LEVELS=0,1,2 KB_LAYERS=0,6,11 timeout -k 10 200 python -u tools/kbench.py > $O/kb_$v.log 2>&1 || exit 1
  grep -v amdgpu $O/kb_$v.log | sed "s/^/$v /"
done
for rep in 1 2; do
for v in dw4 base; do
  if [ $v = base ]; then L=""; else L=tools/ab_lib/$v/libidfcodec.so; fi
  IDF_LIB_PATH=$L timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-residual --no-cpu-baseline > $O/bench_$v.$rep.json 2> $O/bench_$v.$rep.err || exit 1
  python3 -c "import json; d=json.load(open('$O/bench_$v.$rep.json')); print('$v', d['value'], d['serial'], d['roofline']['frac'], d['round_trip_exact_steps'])"
done
done
