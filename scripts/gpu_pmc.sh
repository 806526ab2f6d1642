#!/bin/bash
# PMC counter passes over one short bench run (separate passes, kernel-trace only);
# CONFIG selects the bench --config (c2 by default).
set -u
OUT=${PMC_OUT:-gpurun_out/pmc}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
ARGS="python3 bench.py --config ${CONFIG:-c2} --steps 1 --warmup 1 --no-cpu-baseline --no-regularize"
i=0
for set in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-trace -d $OUT/p$i -o run --output-format csv -- $ARGS \
      > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
ls -R $OUT | head -40
