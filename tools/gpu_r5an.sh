#!/bin/bash
# round 5: wave-priority schedules in the dx3 slab loop (IDF_DX3_PRIO builds) -- kbench L0, bench
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r5an; mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
for v in base pr1 pr2 pr3; do
  if [ $v = base ]; then L=""; else L=tools/ab_lib/$v/libidfcodec.so; fi
  IDF_LIB_PATH=$L KB_B=128 KB_ONLY=dx3 KB_LEVELS=0,1 KB_LAYERS=6,11 timeout -k 10 200 python -u tools/kbench.py > $O/kb_$v.log 2>&1 || exit 1
  grep -v amdgpu $O/kb_$v.log | sed "s/^/$v /"
done
for v in base pr1 pr2 pr3; do
  if [ $v = base ]; then L=""; else L=tools/ab_lib/$v/libidfcodec.so; fi
  IDF_LIB_PATH=$L timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-residual --no-cpu-baseline > $O/bench_$v.json 2> $O/bench_$v.err || exit 1
  python3 -c "import json; d=json.load(open('$O/bench_$v.json')); print('$v', d['value'], d['serial'], d['roofline']['frac'], d['round_trip_exact_steps'])"
done
