#!/bin/bash
# 8x8 / vector epilogue staging-slot swap keyed on the channel: wino tests, LDS conflict
# counters, same-box timing against the previous source (tools/native/wino_base_0), configs 4/5.
set -u -o pipefail
cd "$(dirname "$0")/.."
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/r4i; mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_wino.py \
  tests/test_gpu_production_parity.py -k "wino or wx3 or x3 or config45" > $O/wino_tests.log 2>&1 || { tail -30 $O/wino_tests.log; exit 1; }
tail -1 $O/wino_tests.log
OUT=$O/pmc ABL=0 bash tools/pmc_lds_attr.sh || exit 1
grep -A4 "true, false" $O/pmc/a0.summary
for r in 1 2; do
  for b in wino_base_0 wino_ablate_0; do
    echo "== $b"; timeout -k 10 60 ./tools/native/$b x3 || exit 1
  done
done 2>&1 | grep -v amdgpu.ids | tee $O/ab.txt
for c in resflows_smallpatch_split resflow-patches-vqvae; do
  timeout -k 10 200 python3 -u tools/bench_residual.py --config $c --steps 5 > $O/b_$c.json 2>$O/b_$c.err || { tail -5 $O/b_$c.err; exit 1; }
  cut -c1-300 $O/b_$c.json
done
