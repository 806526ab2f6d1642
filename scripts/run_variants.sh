#!/bin/bash
# Run scripts/score_variants.py once per experiment library (GPU box).
# Usage: scripts/run_variants.sh NAME...   (scripts/exp/libsfm_hip_NAME.so)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for name in "$@"; do
  SFM_HIP_LIB=scripts/exp/libsfm_hip_$name.so timeout -k 10 240 python scripts/score_variants.py \
      >> gpurun_out/variants.log 2>&1 || { echo "variant $name failed ($?)"; tail -5 gpurun_out/variants.log; exit 1; }
done
cat gpurun_out/variants.log
