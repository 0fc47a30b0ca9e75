#!/bin/bash
# round 5: back-to-back encode / decode under lane options (same box, alternating)
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r5o2; mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
for rep in 1 2; do
  for v in "base" "IDF_LANES=4" "IDF_LANES=4 IDF_LANE_STAGGER=levels" "IDF_LANE_SPLIT=0.375 IDF_LANE_STAGGER=levels" "IDF_DECODE_WPB=1"; do
    n=$(echo $v | tr ' =' '__')
    env $([ "$v" = base ] || echo $v) timeout -k 10 200 python -u bench.py --pipeline 0 --steps 6 --warmup 2 --no-residual --no-cpu-baseline > $O/$n.$rep.json 2> $O/$n.$rep.err || exit 1
    python3 -c "import json; d=json.load(open('$O/$n.$rep.json')); print('$v', d['value'], d['encode_ms'], d['decode_ms'])"
  done
done
