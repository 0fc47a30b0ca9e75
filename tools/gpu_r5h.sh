#!/bin/bash
# round 5: decode lane stagger A/B (back-to-back steps), alternating, same box
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r5h; mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
for rep in 1 2; do
  for st in top none flows0 levels; do
    IDF_LANE_STAGGER=$st timeout -k 10 200 python -u bench.py --steps 8 --warmup 2 --pipeline 0 --no-residual \
      --no-cpu-baseline > $O/${st}_$rep.json 2> $O/${st}_$rep.err || exit 1
    python3 -c "import json; d=json.load(open('$O/${st}_$rep.json')); print('$st', $rep, d['value'], d['encode_ms'], d['decode_ms'])"
  done
done
