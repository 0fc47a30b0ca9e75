#!/bin/bash
# Decode lanes vs hardware queues: bench headline (no residual / CPU legs) per setting.
set -u -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/lanes_q
export PYTHONDONTWRITEBYTECODE=1
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --steps 8 --warmup 2 --no-residual --no-cpu-baseline \
    > gpurun_out/lanes_q/$name.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/lanes_q/$name.log; return 1; }
  python3 - "$name" gpurun_out/lanes_q/$name.log <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[2]) if l.startswith("{")][-1]
print(f"{sys.argv[1]:28s} value {d['value']:.3f} enc {d['encode_ms']:.2f} dec {d['decode_ms']:.2f} ms/step {d['ms_per_step']:.2f}")
PY
}
run base IDF_LANES=2 || exit 1
run q8_l2 GPU_MAX_HW_QUEUES=8 IDF_LANES=2 || exit 1
run q8_l4 GPU_MAX_HW_QUEUES=8 IDF_LANES=4 || exit 1
run q8_l4_none GPU_MAX_HW_QUEUES=8 IDF_LANES=4 IDF_LANE_STAGGER=none || exit 1
run q8_l4_levels GPU_MAX_HW_QUEUES=8 IDF_LANES=4 IDF_LANE_STAGGER=levels || exit 1
run q16_l8 GPU_MAX_HW_QUEUES=16 IDF_LANES=8 || exit 1
run q4_l4 IDF_LANES=4 || exit 1
run base2 IDF_LANES=2 || exit 1
