#!/bin/bash
set -u
OUT=gpurun_out/pmc_ta
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
i=0
for cfg in c3 c2; do
for set in "TA_TA_BUSY TA_BUFFER_TOTAL_CYCLES GRBM_GUI_ACTIVE" "TD_TD_BUSY TD_TC_STALL GRBM_GUI_ACTIVE" \
           "TCP_PENDING_STALL_CYCLES TCP_TCP_TA_DATA_STALL_CYCLES TCP_READ_TAGCONFLICT_STALL_CYCLES TCP_TCC_READ_REQ_LATENCY GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $set --kernel-trace -d $OUT/$cfg$i -o run --output-format csv -- python3 bench.py --config $cfg --steps 1 --warmup 1 --no-cpu-baseline --no-regularize \
      > $OUT/$cfg$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/$cfg$i.log; exit 1; }
done
done
echo done
