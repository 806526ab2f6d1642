#!/bin/bash
# Bench every --config once (N=1) after the GPU tests; stops at the first failure.
set -u
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
      ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -15 gpurun_out/pytest_gpu.log
  [ $rc -ne 0 ] && exit $rc
fi
for cfg in ${CONFIGS:-c2 c3 c4 sparse}; do
  extra="--no-cpu-baseline --no-regularize"
  [ "$cfg" = "c2" ] && [ "${C2_FULL:-0}" = "1" ] && extra=""
  timeout -k 10 400 python -u bench.py --config $cfg --steps ${STEPS:-10} --warmup 2 $extra \
      > gpurun_out/bench_$cfg.log 2>&1
  rc=$?; grep '^{' gpurun_out/bench_$cfg.log | cut -c1-600
  [ $rc -ne 0 ] && { tail -20 gpurun_out/bench_$cfg.log; exit $rc; }
done
exit 0
