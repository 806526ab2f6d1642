#!/bin/bash
# rocprofv3 kernel-trace stats of the bench (N=1); CONFIG selects --config.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
cfg=${CONFIG:-c2}
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$cfg -o run --output-format csv -- \
    python3 bench.py --config $cfg --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline --no-regularize \
    > gpurun_out/prof_$cfg.log 2>&1 || exit $?
tail -2 gpurun_out/prof_$cfg.log
find gpurun_out/prof_$cfg -name "*stats*" | head
