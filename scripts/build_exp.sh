#!/bin/bash
# Experiment variants of libsfm_hip.so (score-kernel statistics / no-fallback
# timing) into scripts/exp/, same flags as csrc/Makefile.  Never used by the
# product; selected with SFM_HIP_LIB by scripts/score_experiment.py.
set -e
cd "$(dirname "$0")/../deep-sfm-revisited_amd/csrc"
mkdir -p ../../scripts/exp
for v in STATS NOFALLBACK; do
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math -fno-slp-vectorize -fPIC -shared \
        -I../../include -Wno-unused-result -DSFM_SCORE_$v -o ../../scripts/exp/libsfm_hip_$v.so \
        capi.hip ransac5.hip sweep.hip depth.hip irls.hip host_polish.cpp
done
