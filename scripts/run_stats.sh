#!/bin/bash
# Run scripts/score_experiment.py once per STATS experiment library (GPU box).
# Usage: scripts/run_stats.sh NAME...   (scripts/exp/libsfm_hip_NAME.so)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for name in "$@"; do
  echo "== $name" >> gpurun_out/stats.log
  SFM_HIP_LIB=scripts/exp/libsfm_hip_$name.so timeout -k 10 240 python scripts/score_experiment.py \
      >> gpurun_out/stats.log 2>&1 || { echo "stats $name failed ($?)"; tail -5 gpurun_out/stats.log; exit 1; }
done
grep -v amdgpu.ids gpurun_out/stats.log
