#!/bin/bash
# x3 Winograd conv ablations on the imagenet64 layer shapes (tools/native/wino_ablate_*):
# one run per ablation mask, each under its own time limit.
set -u -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
OUT=gpurun_out/ablate.log
: > $OUT
for a in ${ABL:-0 2 256 59 315 319 47}; do
  timeout -k 10 60 ./tools/native/wino_ablate_$a x3 >> $OUT 2>&1 || exit $?
done
[ -x tools/native/wino_stamps ] && { timeout -k 10 60 ./tools/native/wino_stamps x3 >> $OUT 2>&1 || exit $?; }
cat $OUT
