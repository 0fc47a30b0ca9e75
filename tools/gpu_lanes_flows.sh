#!/bin/bash
# Decode-lane stagger "flows" vs the default: lane tests exact under it, then bench A/B.
set -u -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/lanes_flows
export PYTHONDONTWRITEBYTECODE=1

run() {
  local name=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --steps 12 --warmup 2 --no-residual --no-cpu-baseline \
    > gpurun_out/lanes_flows/$name.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/lanes_flows/$name.log; return 1; }
  python3 - "$name" gpurun_out/lanes_flows/$name.log <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[2]) if l.startswith("{")][-1]
print(f"{sys.argv[1]:14s} value {d['value']:.3f} enc {d['encode_ms']:.2f} dec {d['decode_ms']:.2f} ms/step {d['ms_per_step']:.2f} exact {d['round_trip_exact']}")
PY
}
IDF_LANE_STAGGER=flows0 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_lanes.py > gpurun_out/lanes_flows/tests.log 2>&1 || { tail -30 gpurun_out/lanes_flows/tests.log; exit 1; }
tail -2 gpurun_out/lanes_flows/tests.log
for rep in 1 2 3; do
  run top_$rep IDF_LANE_STAGGER=top || exit 1
  run flows0_$rep IDF_LANE_STAGGER=flows0 || exit 1
done
