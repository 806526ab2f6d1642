#!/bin/bash
# SQ counters of the sweep kernel per tuning variant (GPU box), kernel-trace
# only, one pass per counter set.  Usage: scripts/pmc_sweep.sh "k=v k=v" ...
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/pmcs
export TMPDIR=/tmp
n=0
for variant in "$@"; do
  n=$((n+1))
  i=0
  for set in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES GRBM_GUI_ACTIVE" \
             "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU"; do
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --pmc $set --kernel-trace --kernel-include-regex k_sweep \
        -d gpurun_out/pmcs/v$n/p$i -o run --output-format csv \
        -- python3 scripts/sweep_variant.py $variant > gpurun_out/pmcs/v$n.p$i.log 2>&1 \
        || { echo "pmc variant $n pass $i failed"; tail -5 gpurun_out/pmcs/v$n.p$i.log; exit 1; }
  done
  echo "v$n: $variant" >> gpurun_out/pmcs/variants.txt
done
python3 scripts/pmc_sweep_summary.py
