#!/bin/bash
# conv parity tests + same-box A/B + one LDS-conflict PMC pass of the A/B binaries
set -u -o pipefail
cd "$(dirname "$0")/.."
./tools/gpu_conv.sh && ./tools/gpu_ab.sh || exit $?
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for b in wino_base_0 wino_ablate_0; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS -d gpurun_out/lds_$b -o run --output-format csv -- ./tools/native/$b x3 > gpurun_out/lds_$b.log 2>&1 || exit $?
  python3 tools/pmc_summary.py gpurun_out/lds_$b conv3_wino_kernel > gpurun_out/lds_$b.txt 2>&1
  echo "== $b"; grep -A3 "grid=131072\|grid=524288" gpurun_out/lds_$b.txt | head -16
done
