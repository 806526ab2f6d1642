#!/bin/bash
# One GPU-box session of a round's evidence (tag R, e.g. R=r04): the GPU test
# suite, smoke, the c2 bench line (CPU baseline, regularisation lines),
# rocprofv3 --kernel-trace --stats runs of the c2 / sparse / c3 benches (each
# with its own bench line, which carries the src_hash the profile belongs to),
# the PMC passes of c2 and c3, and the other configs' bench lines.  Stops at
# the first failure.  SKIP_TESTS / SKIP_PROF / SKIP_PMC / SKIP_CONFIGS=1 skip
# a part.  scripts/collect_evidence.py copies the results into profiles/.
set -u
R=${R:-r06}
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
      > gpurun_out/${R}_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/${R}_pytest_gpu.log; exit 1; }
  tail -2 gpurun_out/${R}_pytest_gpu.log
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${R}_smoke.log 2>&1 \
      || { tail -20 gpurun_out/${R}_smoke.log; exit 1; }
  tail -1 gpurun_out/${R}_smoke.log
fi
timeout -k 10 500 python -u bench.py --steps ${STEPS:-20} --warmup 3 > gpurun_out/${R}_bench_c2.log 2>&1 \
    || { tail -20 gpurun_out/${R}_bench_c2.log; exit 1; }
grep '^{' gpurun_out/${R}_bench_c2.log | cut -c1-400
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
if [ "${SKIP_PROF:-0}" != "1" ]; then
  for cfg in c2 sparse c3; do
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${R}_prof_$cfg -o run --output-format csv -- \
        python3 bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline --no-regularize \
        > gpurun_out/${R}_prof_$cfg.log 2>&1 || { tail -20 gpurun_out/${R}_prof_$cfg.log; exit 1; }
    find gpurun_out/${R}_prof_$cfg -name "*kernel_stats*"
  done
fi
if [ "${SKIP_PMC:-0}" != "1" ]; then
  CONFIG=c2 PMC_OUT=gpurun_out/${R}_pmc_c2 timeout -k 10 900 bash scripts/gpu_pmc.sh > gpurun_out/${R}_pmc_c2.log 2>&1 \
      || { tail -20 gpurun_out/${R}_pmc_c2.log; exit 1; }
  CONFIG=c3 PMC_OUT=gpurun_out/${R}_pmc_c3 timeout -k 10 900 bash scripts/gpu_pmc.sh > gpurun_out/${R}_pmc_c3.log 2>&1 \
      || { tail -20 gpurun_out/${R}_pmc_c3.log; exit 1; }
fi
if [ "${SKIP_CONFIGS:-0}" != "1" ]; then
  for cfg in sparse c3 c4 c5; do
    timeout -k 10 300 python -u bench.py --config $cfg --steps 20 --warmup 3 --no-cpu-baseline --no-regularize \
        > gpurun_out/${R}_bench_$cfg.log 2>&1 || { tail -20 gpurun_out/${R}_bench_$cfg.log; exit 1; }
    grep '^{' gpurun_out/${R}_bench_$cfg.log | cut -c1-300
  done
fi
