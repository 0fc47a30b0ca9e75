#!/bin/bash
# Same-box A/B of the decode-lane hold (IDF_LANE_HOLD) on the default bench, plus the host
# enqueue probe and the lanes' exactness tests.
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/hold_ab
mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 240 python3 -u tools/host_issue_probe.py 2>&1 | grep -v amdgpu.ids > $O/host_probe.log || exit $?
cat $O/host_probe.log
for r in 1 2; do
  for h in 0 2 4 6; do
    IDF_LANE_HOLD=$h timeout -k 10 180 python3 -u bench.py --no-residual --no-cpu-baseline --steps 10 --warmup 2 2>/dev/null > $O/b_${h}_$r.json || exit $?
    python3 -c "import json,sys; d=json.load(open('$O/b_${h}_$r.json')); print('hold $h', d['value'], 'enc', d['encode_ms'], 'dec', d['decode_ms'], 'exact', d['round_trip_exact'])"
  done
done | tee $O/summary.txt
IDF_LANE_HOLD=4 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_lanes.py > $O/lanes_tests.log 2>&1; tail -2 $O/lanes_tests.log
