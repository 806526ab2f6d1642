#!/bin/bash
# One GPU-box session of round-3 evidence: the GPU test suite, smoke, the c2
# bench line (CPU baseline, regularisation lines), a rocprofv3 kernel-trace
# --stats run of the same bench (its own bench line kept beside the CSV), the
# PMC passes, and the other configs' bench lines.  Stops at the first failure.
set -u
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
      > gpurun_out/r3_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r3_pytest_gpu.log; exit 1; }
  tail -2 gpurun_out/r3_pytest_gpu.log
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_smoke.log 2>&1 \
      || { tail -20 gpurun_out/r3_smoke.log; exit 1; }
  tail -1 gpurun_out/r3_smoke.log
fi
timeout -k 10 500 python -u bench.py --steps ${STEPS:-20} --warmup 3 > gpurun_out/r3_bench_c2.log 2>&1 \
    || { tail -20 gpurun_out/r3_bench_c2.log; exit 1; }
grep '^{' gpurun_out/r3_bench_c2.log | cut -c1-400
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r3_prof_c2 -o run --output-format csv -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-regularize > gpurun_out/r3_prof_c2.log 2>&1 \
    || { tail -20 gpurun_out/r3_prof_c2.log; exit 1; }
find gpurun_out/r3_prof_c2 -name "*kernel_stats*"
if [ "${SKIP_PMC:-0}" != "1" ]; then
  CONFIG=c2 timeout -k 10 900 bash scripts/gpu_pmc.sh > gpurun_out/r3_pmc.log 2>&1 || { tail -20 gpurun_out/r3_pmc.log; exit 1; }
fi
if [ "${SKIP_PMC:-0}" != "1" ]; then
  CONFIG=c3 PMC_OUT=gpurun_out/pmc_c3 timeout -k 10 900 bash scripts/gpu_pmc.sh > gpurun_out/r3_pmc_c3.log 2>&1 \
      || { tail -20 gpurun_out/r3_pmc_c3.log; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3_prof_c3 -o run --output-format csv -- \
      python3 bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline --no-regularize \
      > gpurun_out/r3_prof_c3.log 2>&1 || { tail -20 gpurun_out/r3_prof_c3.log; exit 1; }
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3_prof_sparse -o run --output-format csv -- \
    python3 bench.py --config sparse --steps 10 --warmup 2 --no-cpu-baseline --no-regularize \
    > gpurun_out/r3_prof_sparse.log 2>&1 || { tail -20 gpurun_out/r3_prof_sparse.log; exit 1; }
for cfg in sparse c3 c4; do
  timeout -k 10 300 python -u bench.py --config $cfg --steps 20 --warmup 3 --no-cpu-baseline --no-regularize \
      > gpurun_out/r3_bench_$cfg.log 2>&1 || { tail -20 gpurun_out/r3_bench_$cfg.log; exit 1; }
  grep '^{' gpurun_out/r3_bench_$cfg.log | cut -c1-300
done
