#!/bin/bash
# 2 vs 3 decode lanes at batch 258 (divisible by both), alternated
set -u -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
for n in 2 3 2 3; do
  IDF_LANES=$n timeout -k 10 300 python -u bench.py --no-residual --no-cpu-baseline --steps 5 --batch 258 > gpurun_out/lanes3_b.log 2>&1 || { tail -20 gpurun_out/lanes3_b.log; exit 1; }
  echo "lanes=$n $(python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/lanes3_b.log') if l.startswith('{')][-1]); print(d['value'], 'enc', d['encode_ms'], 'dec', d['decode_ms'], 'exact', d['round_trip_exact'])")"
done
