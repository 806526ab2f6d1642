#!/bin/bash
# SQ issue counters of the sweep kernels (k_sweep_tile vs k_sweep_band), fp32
# and bf16, two kernel-trace-only passes per variant (GPU box).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/pmcs
export TMPDIR=/tmp
for var in "flat2:sweep_flat=2" "band16:sweep_flat=3 sweep_run=16" "band32:sweep_flat=3 sweep_run=32" \
           "flat2bf:sweep_flat=2 dtype=bf16" "band32bf:sweep_flat=3 sweep_run=32 dtype=bf16"; do
  name=${var%%:*}; args=${var#*:}
  i=0
  for set in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
             "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_WR"; do
    i=$((i+1))
    # shellcheck disable=SC2086
    timeout -k 10 120 rocprofv3 --pmc $set --kernel-trace --kernel-include-regex k_sweep \
        -d gpurun_out/pmcs/$name/p$i -o run --output-format csv \
        -- python3 scripts/sweep_variant.py $args > gpurun_out/pmcs/$name.p$i.log 2>&1 \
        || { echo "pmc $name pass $i failed"; tail -5 gpurun_out/pmcs/$name.p$i.log; exit 1; }
  done
done
python3 scripts/pmc_sweep_sq_summary.py flat2 band16 band32 flat2bf band32bf
