#!/bin/bash
# Round 4: the N=2 rehearsal of the pipelined bench (2 ranks on cuda:0 over gloo), then the
# whole GPU suite + smoke at HEAD.
set -u -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r4f; mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
IDF_DIST_BACKEND=gloo IDF_SHARE_GPU=1 IDF_DIST_HOST_GROUP=separate timeout -k 10 400 python -u bench.py --gpus 2 --steps 3 --warmup 1 \
  --no-cpu-baseline --no-residual > $O/rh2.log 2>&1 || { tail -30 $O/rh2.log; exit 1; }
tail -1 $O/rh2.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("N=2 rehearsal", d["value"], d["pipelined"], "exact", d["round_trip_exact"], "gathered", d["gathered_bitstream_exact"])'
O=$O bash tools/gpu_r3_final_a.sh
