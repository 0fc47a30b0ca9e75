#!/bin/bash
# round 5: slab-major dxb + fused head -- tests, config 3 A/B, kbench
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r5s; mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_lanes.py -k "dxb or bf16 or two_streams" -x -q --timeout 200 --timeout-method thread > $O/t.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/t.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_production_parity.py -x -q --timeout 300 --timeout-method thread -s -k "config3" > $O/cfg3.log 2>&1
rc=$?; echo "cfg3 rc=$rc"; grep -E "config 3|passed|failed|Error" $O/cfg3.log | tail -6; [ $rc -ne 0 ] && exit $rc
KB_B=1024 KB_ONLY=dxb KB_LEVELS=0,1,2 KB_LAYERS=0,3,6,9,11 timeout -k 10 200 python -u tools/kbench.py > $O/kb.log 2>&1 || exit 1
grep -v amdgpu $O/kb.log
for v in 1 0; do
  IDF_DXB=$v timeout -k 10 300 python -u tools/bench_residual.py --config resflow-cond-imagenet64 > $O/res_dxb$v.json 2> $O/res_dxb$v.err || exit 1
  python3 -c "import json; d=json.load(open('$O/res_dxb$v.json')); r=d.get('roofline', {}); print('IDF_DXB=$v', d.get('value'), d.get('encode_ms'), d.get('decode_ms'), r.get('frac'), r.get('avg_launch_ms'), r.get('conv_mode'))"
done
