#!/bin/bash
# VQ argmin: exactness tests, then timing at the residual configs' shapes and configs 4/5.
set -u -o pipefail
cd "$(dirname "$0")/.."
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/vq; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_vq.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 120 python3 -u tools/vq_argmin_bench.py 2>&1 | grep -v amdgpu.ids | tee $O/bench.txt
for c in resflows_smallpatch_split resflow-patches-vqvae; do
  timeout -k 10 200 python3 -u tools/bench_residual.py --config $c --steps 5 > $O/b_$c.json 2>$O/b_$c.err || { tail -5 $O/b_$c.err; exit 1; }
  cut -c1-330 $O/b_$c.json
done
