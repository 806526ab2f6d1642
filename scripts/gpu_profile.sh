#!/bin/bash
# rocprofv3 kernel-trace stats of the bench (N=1).
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o run --output-format csv -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1 || exit $?
tail -2 gpurun_out/prof_bench.log
find gpurun_out/prof_bench -name "*stats*" | head
