#!/bin/bash
# PMC passes over the regularisation stack (scripts/bench_regularize.py --steps 1), kernel-trace only.
mkdir -p gpurun_out/pmc_conv
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
i=0
for set in "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM_RD" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace -d gpurun_out/pmc_conv/p$i -o run --output-format csv -- \
      python3 scripts/bench_regularize.py --steps 1 > gpurun_out/pmc_conv/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc_conv/p$i.log; exit 1; }
done
echo ok
