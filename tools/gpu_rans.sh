#!/bin/bash
# rANS GPU step: the rANS parity tests, then the decode/encode timing harness at 3072 and
# 6144 symbols per stream (tools/native/rans_bench_0).
set -u -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_rans.py > gpurun_out/rans_tests.log 2>&1; rc=$?
tail -30 gpurun_out/rans_tests.log
[ $rc -eq 0 ] || exit $rc
for n in 3072 6144; do
  timeout -k 10 60 ./tools/native/rans_bench_0 $n >> gpurun_out/rans_bench.log 2>&1 || exit $?
done
cat gpurun_out/rans_bench.log
