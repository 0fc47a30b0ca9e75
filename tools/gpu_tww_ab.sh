#!/bin/bash
# 16x16 vs 32x8 output tiles for images wider than 32 (the VQ-VAE convs): VQ/residual parity with
# 16, then a same-box A/B of the residual configs.
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/tww
mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
IDF_WINO_TWW=16 timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_vq.py tests/test_gpu_residual.py tests/test_gpu_wx3.py tests/test_gpu_wino.py > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for t in 16 32; do
    for c in resflow-cond-imagenet64 resflows_smallpatch_split resflow-patches-vqvae; do
      IDF_WINO_TWW=$t timeout -k 10 300 python3 -u tools/bench_residual.py --config $c --steps 3 --warmup 1 2>/dev/null | tail -1 > $O/r_${t}_${c}_$r.json || exit $?
      python3 -c "import json; d=json.load(open('$O/r_${t}_${c}_$r.json')); print('tww $t $c', d.get('value'), d.get('encode_ms'), d.get('decode_ms'))"
    done
  done
done | tee $O/summary.txt
