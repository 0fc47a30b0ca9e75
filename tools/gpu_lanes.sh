#!/bin/bash
# decode-lane ordering A/B: lane tests, then bench under each IDF_LANE_STAGGER / IDF_LANE_PRIO
set -u -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_lanes.py > gpurun_out/lanes_tests.log 2>&1 || { tail -20 gpurun_out/lanes_tests.log; exit 1; }
tail -2 gpurun_out/lanes_tests.log
for v in "top 0.5" "top 0.4375" "top 0.40625" "levels 0.4375" "top 0.375" "top 0.5"; do
  set -- $v
  IDF_LANE_STAGGER=$1 IDF_LANE_SPLIT=$2 timeout -k 10 300 python -u bench.py --no-residual --no-cpu-baseline --steps 5 > gpurun_out/lanes_b.log 2>&1 || { tail -20 gpurun_out/lanes_b.log; exit 1; }
  echo "stagger=$1 split=$2 $(python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/lanes_b.log') if l.startswith('{')][-1]); print(d['value'], 'enc', d['encode_ms'], 'dec', d['decode_ms'])")"
done
