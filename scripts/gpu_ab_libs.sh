#!/bin/bash
# Score-kernel A/B across library builds (scripts/build_exp.sh NAME=FLAGS ...):
# each library in its own process, alternating, ROUNDS rounds; then each
# STATS library once for its undecided fraction.  Usage:
#   LIBS="D6 prod D4" STATS="D6S D5S" ROUNDS=2 bash scripts/gpu_ab_libs.sh
# ("prod" = the in-tree libsfm_hip.so).  Stops at the first failure.
set -u
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
lib() { if [ "$1" = prod ]; then echo deep-sfm-revisited_amd/sfm_amd/libsfm_hip.so; else echo ${EXPDIR:-scripts/exp}/libsfm_hip_$1.so; fi; }
for r in $(seq 1 ${ROUNDS:-2}); do
  for L in ${LIBS}; do
    echo "== round $r lib $L"
    SFM_HIP_LIB=$(lib $L) timeout -k 10 180 python -u scripts/mf2_ab.py ${AB_ARGS:-} || exit 1
  done
done
for L in ${STATS:-}; do
  echo "== stats lib $L"
  SFM_HIP_LIB=$(lib $L) timeout -k 10 180 python -u scripts/mf2_ab.py ${AB_ARGS:-} || exit 1
done
