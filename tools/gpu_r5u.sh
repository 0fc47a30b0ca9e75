#!/bin/bash
# round 5: split-K chunks at the 8x8 level (timing A/B builds), bench + 8x8 kbench
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r5u; mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
for rep in 1 2; do
for v in base ks2 ks3; do
  if [ $v = base ]; then L=""; else L=tools/ab_lib/$v/libidfcodec.so; fi
  IDF_LIB_PATH=$L timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-residual --no-cpu-baseline > $O/bench_$v.$rep.json 2> $O/bench_$v.$rep.err || exit 1
  python3 -c "import json; d=json.load(open('$O/bench_$v.$rep.json')); print('$v', d['value'], d['serial'], d['roofline']['frac'])"
done
done
for v in base ks2 ks3; do
  if [ $v = base ]; then L=""; else L=tools/ab_lib/$v/libidfcodec.so; fi
  IDF_LIB_PATH=$L KB_ONLY=dx3 KB_LEVELS=2 KB_LAYERS=0,3,6,9,11 KB_B=128 timeout -k 10 200 python -u tools/kbench.py 2>&1 | grep -v amdgpu | sed "s/^/$v /"
done
