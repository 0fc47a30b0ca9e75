#!/bin/bash
# Round 3: VQ-VAE ResBlock convs on split-f16 Winograd -- parity tests, then configs 4/5 A/B.
set -u -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_vq.py tests/test_gpu_residual.py > gpurun_out/r3b_tests.log 2>&1 || {
  tail -c 4000 gpurun_out/r3b_tests.log; exit 1; }
tail -n 3 gpurun_out/r3b_tests.log
for cfg in resflows_smallpatch_split resflow-patches-vqvae resflow-cond-imagenet64; do
  for m in x3 f32; do
    IDF_VQ_CONV=$m timeout -k 10 300 python -u tools/bench_residual.py --config $cfg --steps 3 \
      > gpurun_out/r3b_${cfg}_$m.json 2> gpurun_out/r3b_${cfg}_$m.err || { tail -c 2000 gpurun_out/r3b_${cfg}_$m.err; exit 1; }
    echo "$cfg $m: $(cat gpurun_out/r3b_${cfg}_$m.json)"
  done
done
