#!/bin/bash
# GPU box: regularisation parity tests, then the stack timing (scripts/bench_regularize.py).
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_regularize.py -v --timeout 120 --timeout-method thread > gpurun_out/reg_tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|assert" gpurun_out/reg_tests.log | tail -30
[ $rc -le 1 ] || exit $rc
echo "== default"; timeout -k 10 120 python scripts/bench_regularize.py || exit $?
for v in ${VARIANTS:-}; do echo "== $v"; SFM_HIP_LIB=scripts/exp/libsfm_hip_$v.so timeout -k 10 120 python scripts/bench_regularize.py || exit $?; done
