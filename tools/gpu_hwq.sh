#!/bin/bash
# HIP hardware queues per process for the pipelined bench (bench.py sets 8 unless given).
set -u -o pipefail
cd "$(dirname "$0")/.."
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/hwq; mkdir -p $O
for r in 1 2 3; do
  for q in ${HWQ_VARIANTS:-8 16 4}; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python3 -u bench.py --no-residual --no-cpu-baseline --steps 10 --warmup 2 > $O/b_${q}_$r.json 2>$O/err.log || { tail -5 $O/err.log; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b_${q}_$r.json')); print('hwq $q', d['value'], 'enc', d['encode_ms'], 'dec', d['decode_ms'], 'exact', d['round_trip_exact'])"
  done
done | tee $O/ab.txt
