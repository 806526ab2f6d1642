#!/bin/bash
# SQ counters of one kernel (regex $1) over `python3 scripts/score_knobs.py <knobs>`
# per variant, one pass per counter set (kernel-trace only).
# Usage: scripts/pmc_kernel.sh REGEX "k=v k=v" ...
set -o pipefail
cd "$(dirname "$0")/.."
re=$1; shift
mkdir -p gpurun_out/pmck
export TMPDIR=/tmp
n=0
: > gpurun_out/pmck/variants.txt
for variant in "$@"; do
  n=$((n+1))
  i=0
  for set in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE" \
             "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INST_CYCLES_SALU"; do
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --pmc $set --kernel-trace --kernel-include-regex "$re" \
        -d gpurun_out/pmck/v$n/p$i -o run --output-format csv \
        -- python3 scripts/score_knobs.py $variant > gpurun_out/pmck/v$n.p$i.log 2>&1 \
        || { echo "pmc variant $n pass $i failed"; tail -5 gpurun_out/pmck/v$n.p$i.log; exit 1; }
  done
  echo "v$n: $variant" >> gpurun_out/pmck/variants.txt
done
python3 scripts/pmc_kernel_summary.py "$re"
