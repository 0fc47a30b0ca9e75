#!/bin/bash
# NF=2 compile-time tile widths (wx3 TWC 32/16/8/24): tests, then same-box A/B of the residual
# configs against the previous library (tools/ab_lib/prev).
set -u -o pipefail
cd "$(dirname "$0")/.."
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/r4j; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_wino.py \
  tests/test_gpu_vq.py tests/test_gpu_residual.py tests/test_gpu_production_parity.py -k "not config3_full" \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in prev new; do
    lp=""; [ $v = prev ] && lp=$PWD/tools/ab_lib/prev/libidfcodec.so
    for c in resflows_smallpatch_split resflow-patches-vqvae resflow-cond-imagenet64; do
      IDF_LIB_PATH=$lp timeout -k 10 300 python3 -u tools/bench_residual.py --config $c --steps 4 > $O/b_${v}_${c}_$r.json 2>$O/err.log || { tail -5 $O/err.log; exit 1; }
      python3 -c "import json; d=json.load(open('$O/b_${v}_${c}_$r.json')); print('$v', '$c', d['value'], 'enc', d['encode_ms'], 'dec', d['decode_ms'], 'vq', d['vq_indices_ms'], d['vq_reconstruct_ms'], 'frac', d['roofline']['frac'], d['round_trip_exact'])"
    done
  done
done | tee $O/ab.txt
