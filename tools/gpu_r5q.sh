#!/bin/bash
# round 5: the bf16 direct conv (dxb) -- kernel tests, config 3 teacher-forced blocks and
# round trips, dx3 kernel tests unchanged, then config 3 throughput dxb vs bf16 (same box)
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r5q; mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
for v in 1 0 1 0; do
  IDF_DXB=$v timeout -k 10 300 python -u tools/bench_residual.py --config resflow-cond-imagenet64 > $O/res_dxb$v.json 2> $O/res_dxb$v.err || exit 1
  python3 -c "import json; d=json.load(open('$O/res_dxb$v.json')); r=d.get('roofline', {}); print('IDF_DXB=$v', d.get('value'), r.get('frac'), r.get('avg_launch_ms'), r.get('conv_mode'))"
done
