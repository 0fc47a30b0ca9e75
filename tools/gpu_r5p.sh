#!/bin/bash
# round 5: the bf16 direct conv (dxb) -- kernel tests, config 3 teacher-forced blocks and
# round trips, dx3 kernel tests unchanged, then config 3 throughput dxb vs bf16 (same box)
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r5p; mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16.py -x -v --timeout 200 --timeout-method thread -s > $O/bf16_tests.log 2>&1
rc=$?; echo "bf16 tests rc=$rc"; grep -E "PASS|FAIL|Error|error" $O/bf16_tests.log | tail -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_production_parity.py -x -q --timeout 300 --timeout-method thread -s -k "config3" > $O/cfg3.log 2>&1
rc=$?; echo "cfg3 rc=$rc"; grep -E "config 3|passed|failed|Error" $O/cfg3.log | tail -8
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_dx3.py -x -q --timeout 120 --timeout-method thread > $O/dx3.log 2>&1
rc=$?; echo "dx3 rc=$rc"; tail -1 $O/dx3.log
[ $rc -ne 0 ] && exit $rc
for v in 1 0 1 0; do
  IDF_DXB=$v timeout -k 10 300 python -u tools/bench_residual.py --config resflow-cond-imagenet64 > $O/res_dxb$v.json 2> $O/res_dxb$v.err || exit 1
  python3 -c "import json; d=json.load(open('$O/res_dxb$v.json')); r=d.get('roofline', {}); print('IDF_DXB=$v', d.get('value'), r.get('frac'), r.get('avg_launch_ms'), r.get('conv_mode'))"
done
