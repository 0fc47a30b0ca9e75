#!/bin/bash
# One-GPU rehearsal of the bench's N-rank path: 2 ranks on cuda:0, collectives over gloo
# staged through host memory (the driver's real N-GPU run uses RCCL, one GPU per rank).
set -u -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5rh
export PYTHONDONTWRITEBYTECODE=1
IDF_DIST_BACKEND=gloo IDF_SHARE_GPU=1 IDF_DIST_HOST_GROUP=separate timeout -k 10 900 python -u bench.py --gpus 2 --steps 3 --warmup 1 \
  --no-cpu-baseline > gpurun_out/r5rh/rh2.log 2>&1; rc=$?
tail -c 3000 gpurun_out/r5rh/rh2.log
exit $rc
