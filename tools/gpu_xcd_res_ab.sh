#!/bin/bash
# XCD-aware order in the bf16 conv (config 3) and the VQ-VAE tap convs (configs 3-5): parity,
# then a same-box A/B of the residual configs against a build with every XCD remap off.
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/xcd_res
mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bf16.py tests/test_gpu_vq.py tests/test_gpu_residual.py > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -ne 0 ] && exit $rc
T=finalproject-losslessimagecompression_amd/idfcodec/libidfcodec.so
for r in 1 2; do
  for v in on off; do
    if [ $v = on ]; then L=$T; else L=tools/xcd_lib/off/libidfcodec.so; fi
    for c in resflow-cond-imagenet64 resflows_smallpatch_split resflow-patches-vqvae; do
      IDF_LIB_PATH=$L timeout -k 10 300 python3 -u tools/bench_residual.py --config $c --steps 3 --warmup 1 2>/dev/null | tail -1 > $O/r_${v}_${c}_$r.json || exit $?
      python3 -c "import json; d=json.load(open('$O/r_${v}_${c}_$r.json')); print('xcd $v $c', d.get('value'), d.get('encode_ms'), d.get('decode_ms'))"
    done
  done
done | tee $O/summary.txt
