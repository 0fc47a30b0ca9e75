#!/bin/bash
# (A/B record: tools/ab_lib/prev was the library before a streaming head-GEMM experiment,
# since reverted; results in profiles/r04/head_gemm/.)
set -u -o pipefail
cd "$(dirname "$0")/.."
export PYTHONDONTWRITEBYTECODE=1
for v in prev new prev new; do
  lp=""; [ $v = prev ] && lp=$PWD/tools/ab_lib/prev/libidfcodec.so
  echo "== $v"; IDF_LIB_PATH=$lp timeout -k 10 120 python3 -u tools/head_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
done
