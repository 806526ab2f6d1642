#!/bin/bash
# One GPU-box session: parity tests, smoke, bench.  Stops at the first crash,
# abort or timeout (exit codes other than 0 = pass, 1 = test failures).
set -u
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 ${T_TEST:-900} python -m pytest tests -m gpu -q -p no:cacheprovider ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest crashed/timeout rc=$rc"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
src=$?
cat gpurun_out/smoke.log | tail -5
if [ $src -ne 0 ] && [ $src -ne 1 ]; then echo "smoke crashed rc=$src"; exit $src; fi
if [ "${SKIP_BENCH:-0}" = "1" ]; then exit $rc; fi
timeout -k 10 ${T_BENCH:-600} python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
brc=$?
tail -5 gpurun_out/bench.log
exit $(( rc | src | brc ))
