#!/bin/bash
# parity tests, then the residual configs' bench (tools/bench_residual.py) twice each
set -u -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu "$@" \
    > gpurun_out/res_ab_tests.log 2>&1; rc=$?; tail -3 gpurun_out/res_ab_tests.log; [ $rc -eq 0 ] || exit $rc
fi
for c in resflow-patches-vqvae resflows_smallpatch_split resflow-patches-vqvae resflows_smallpatch_split; do
  timeout -k 10 300 python -u tools/bench_residual.py --config $c --steps 3 --warmup 1 > gpurun_out/res_b.log 2>&1 || { tail -20 gpurun_out/res_b.log; exit 1; }
  echo "$c: $(tail -1 gpurun_out/res_b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["encode_ms"], d["decode_ms"], d["round_trip_exact"])')"
done
