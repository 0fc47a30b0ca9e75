#!/bin/bash
# Round-4 evidence, part B: the default bench line, its rocprofv3 kernel stats, and the PMC
# traffic passes of the headline bench (tools/pmc_bench.sh, tied to the conv source hash).
set -u -o pipefail
cd "$(dirname "$0")/.."
O=${O:-gpurun_out/r4final2}
O=$O bash tools/gpu_r3_final_b.sh || exit 1
bash tools/pmc_bench.sh || exit 1
