#!/bin/bash
# round 5: the slab's first DMA piece at step 2 / 3 (IDF_DX3_DMA0 builds) now that the first
# fragment reads go first -- kbench and bench A/B against the library (step 0)
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r5at; mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
for v in d2 d3 base; do
  if [ $v = base ]; then L=""; else L=tools/ab_lib/$v/libidfcodec.so; fi
  IDF_LIB_PATH=$L KB_B=128 KB_ONLY=dx3 KB_LEVELS=0,1,2 KB_LAYERS=6,11 timeout -k 10 200 python -u tools/kbench.py > $O/kb_$v.log 2>&1 || exit 1
  grep -v amdgpu $O/kb_$v.log | sed "s/^/$v /"
done
for rep in 1 2; do
for v in d2 d3 base; do
  if [ $v = base ]; then L=""; else L=tools/ab_lib/$v/libidfcodec.so; fi
  IDF_LIB_PATH=$L timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-residual --no-cpu-baseline > $O/bench_$v.$rep.json 2> $O/bench_$v.$rep.err || exit 1
  python3 -c "import json; d=json.load(open('$O/bench_$v.$rep.json')); print('$v', d['value'], d['serial'], d['roofline']['frac'], d['round_trip_exact_steps'])"
done
done
