#!/bin/bash
# One GPU-box session for round-4 iteration: the parity tests named in TESTS
# (default: the scorer / RANSAC set), then a library A/B of the score kernel
# (LIBS / STATS as scripts/gpu_ab_libs.sh).  Stops at the first crash or timeout.
set -u
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
TESTS=${TESTS-"tests/test_gpu_score_mf.py tests/test_gpu_score_edge.py tests/test_gpu_large_n.py tests/test_gpu_ransac.py tests/test_gpu_prune.py"}
if [ -n "$TESTS" ]; then
  timeout -k 10 ${T_TEST:-700} python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
      ${PYTEST_ARGS:-} $TESTS > gpurun_out/s_tests.log 2>&1
  rc=$?; tail -8 gpurun_out/s_tests.log
  [ $rc -ne 0 ] && exit $rc
fi
if [ -n "${LIBS:-}" ]; then
  rm -f gpurun_out/ab_ref.pt
  if [ "${NOREF:-0}" = "1" ]; then REFV=""; export AB_NOCHECK=1; else REFV=gpurun_out/ab_ref.pt; fi   # NOREF: timing-only builds
  AB_REF=$REFV bash scripts/gpu_ab_libs.sh > gpurun_out/s_ab.log 2>&1
  rc=$?; grep -E "==|median|undecided|equal|Error|error" gpurun_out/s_ab.log; exit $rc
fi
