#!/bin/bash
# rANS decode: parity tests, then same-box A/B of the serial decode (tools/native/rans_bench_0
# = current source, rans_base_0 = the saved baseline copy), alternating.
set -u -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/rans_ab
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_rans.py \
  > gpurun_out/rans_ab/tests.log 2>&1 || { tail -30 gpurun_out/rans_ab/tests.log; exit 1; }
tail -1 gpurun_out/rans_ab/tests.log
for rep in 1 2 3; do
  for b in rans_base_0 rans_bench_0; do
    for n in 3072 6144; do
      echo "$b $n: $(timeout -k 10 60 ./tools/native/$b $n | grep mode=)" || exit 1
    done
  done
done 2>&1 | tee gpurun_out/rans_ab/ab.txt
