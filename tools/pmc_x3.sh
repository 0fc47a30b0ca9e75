set -e
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
mkdir -p gpurun_out/pmc_x3
for c in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU" "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_BUSY_CYCLES"; do
  n=$(echo $c | cut -d' ' -f1)
  timeout -s KILL 90 rocprofv3 --pmc $c -d gpurun_out/pmc_x3/$n -o run --output-format csv -- ./tools/native/wino_ablate_0 x3 > gpurun_out/pmc_x3/$n.log 2>&1
done
