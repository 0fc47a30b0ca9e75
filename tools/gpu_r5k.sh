#!/bin/bash
# round 5: the fused head -- kernel tests, teacher-forced blocks (imagenet64 all levels, configs
# 4/5), codec / lanes / B=256 streams vs the oracle, then the bench and a kernel-stats profile
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r5k; mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_dx3.py -x -q --timeout 120 --timeout-method thread -s \
  > $O/dx3_tests.log 2>&1
rc=$?; echo "dx3 tests rc=$rc"; grep -E "fused head|passed|failed|Error" $O/dx3_tests.log | tail -8
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_production_parity.py tests/test_gpu_codec.py \
  tests/test_gpu_lanes.py tests/test_gpu_flow.py -x -q --timeout 300 --timeout-method thread -s \
  -k "teacher_forced or config45 or b256 or conv_modes or guard or lanes or beside or flips or forward_vs" \
  > $O/parity.log 2>&1
rc=$?; echo "parity rc=$rc"; grep -E "worst|flips|passed|failed|Error" $O/parity.log | tail -16
[ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python -u bench.py --steps 10 --warmup 2 --no-residual --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 1
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['serial'], d['round_trip_exact_steps'], d['roofline']['frac'], d['roofline']['avg_launch_ms'])"
O=$O/prof ./tools/gpu_prof.sh > /dev/null 2>&1 || exit 1
head -12 $O/prof/kernel_stats.csv | cut -d, -f1-4
