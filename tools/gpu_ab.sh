#!/bin/bash
# A/B of a bit-identical performance switch: parity tests first, then alternating bench runs.
# usage: tools/gpu_ab.sh "ENV=0" "ENV=1" [test files...]
set -u -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
A=$1; B=$2; shift 2
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu "$@" \
    > gpurun_out/ab_tests.log 2>&1; rc=$?; tail -3 gpurun_out/ab_tests.log; [ $rc -eq 0 ] || exit $rc
fi
for v in "$A" "$B" "$A" "$B"; do
  env $v timeout -k 10 300 python bench.py --no-cpu-baseline --no-residual --steps 10 --warmup 2 \
    > gpurun_out/ab_b.log 2>&1 || { tail -20 gpurun_out/ab_b.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/ab_b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["encode_ms"], d["decode_ms"], d["round_trip_exact"], d["roofline"]["frac"])')"
done
