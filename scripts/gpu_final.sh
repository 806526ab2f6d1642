#!/bin/bash
# One GPU-box session for a round's final evidence: the GPU test suite, smoke,
# the bench lines (c2 with CPU baseline and regularisation line, sparse, c3)
# and rocprofv3 kernel-trace stats of the c2 bench.  Stops at the first failure.
set -u
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
    || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
for cfg in c2 sparse c3; do
  extra="--no-cpu-baseline --no-regularize"
  [ "$cfg" = "c2" ] && extra=""
  timeout -k 10 400 python -u bench.py --config $cfg --steps ${STEPS:-20} --warmup 3 $extra \
      > gpurun_out/bench_$cfg.log 2>&1 || { tail -20 gpurun_out/bench_$cfg.log; exit 1; }
  grep '^{' gpurun_out/bench_$cfg.log | cut -c1-300
done
CONFIG=c2 STEPS=5 bash scripts/gpu_profile.sh
