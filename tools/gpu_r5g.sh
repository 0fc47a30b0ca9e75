#!/bin/bash
# round 5: gutter packing -- dx3 parity, configs 4/5 blocks teacher-forced, then configs 4/5
# conv kernels dx3 vs wx3 (rocprofv3 kernel stats)
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r5g; mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_dx3.py -x -q --timeout 120 --timeout-method thread \
  > $O/dx3_tests.log 2>&1
rc=$?; echo "dx3 tests rc=$rc"; tail -4 $O/dx3_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_production_parity.py -x -v --timeout 300 \
  --timeout-method thread -k "config45" -s > $O/parity.log 2>&1
rc=$?; echo "parity rc=$rc"; grep -E "worst|passed|failed|Error" $O/parity.log | tail -8
[ $rc -ne 0 ] && exit $rc
R=$(pwd); cd /tmp && export TMPDIR=/tmp && cd "$R"
for c in resflows_smallpatch_split resflow-patches-vqvae; do
  for m in dx3 wx3; do
    if [ $m = wx3 ]; then export IDF_DX3=0; else unset IDF_DX3; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p -o run --output-format csv -- \
      python3 -u tools/bench_residual.py --config $c --steps 2 > $O/${c}_$m.json 2> $O/${c}_$m.err || exit 1
    f=$(ls $O/p/*kernel_stats.csv $O/p/*/*kernel_stats.csv 2>/dev/null | head -1); cp "$f" $O/${c}_$m.csv; rm -rf $O/p
    tail -1 $O/${c}_$m.json | cut -c1-150
  done
done
