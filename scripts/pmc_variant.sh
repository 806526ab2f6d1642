#!/bin/bash
# SQ counters of the score kernel for experiment builds (GPU box), two passes
# each (kernel-trace only).  Usage: scripts/pmc_variant.sh NAME...
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/pmcv
export TMPDIR=/tmp
for name in "$@"; do
  i=0
  for set in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD" \
             "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU"; do
    i=$((i+1))
    SFM_HIP_LIB=scripts/exp/libsfm_hip_$name.so timeout -k 10 300 rocprofv3 --pmc $set --kernel-trace \
        --kernel-include-regex k_score32 -d gpurun_out/pmcv/$name/p$i -o run --output-format csv \
        -- python3 scripts/score_variants.py > gpurun_out/pmcv/$name.p$i.log 2>&1 \
        || { echo "pmc $name pass $i failed"; tail -5 gpurun_out/pmcv/$name.p$i.log; exit 1; }
  done
done
python3 scripts/pmc_variant_summary.py "$@"
