#!/bin/bash
# round 5: fused head A/B on one box -- bench (serial encode / decode split) with the fused head
# and with the GEMM heads (IDF_HEAD_FUSE=0), twice each, then kernel stats of both
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r5l; mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
for rep in 1 2; do
  for f in 1 0; do
    IDF_HEAD_FUSE=$f timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-residual --no-cpu-baseline > $O/bench_f${f}_$rep.json 2> $O/bench_f${f}_$rep.err || exit 1
    python3 -c "import json; d=json.load(open('$O/bench_f${f}_$rep.json')); print('fuse $f', d['value'], d['serial'], d['roofline']['frac'], d['roofline']['avg_launch_ms'])"
  done
done
IDF_HEAD_FUSE=1 O=$O/prof1 ./tools/gpu_prof.sh > /dev/null 2>&1 || exit 1
IDF_HEAD_FUSE=0 O=$O/prof0 ./tools/gpu_prof.sh > /dev/null 2>&1 || exit 1
echo ok
