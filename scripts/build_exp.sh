#!/bin/bash
# Experiment variants of libsfm_hip.so into scripts/exp/ (same flags as
# csrc/Makefile); never used by the product, selected with SFM_HIP_LIB.
# With no arguments builds the standard set:
#   STATS       score-kernel undecided statistics   (scripts/score_experiment.py)
#   SOLVESTATS  per-phase cycle counters of k_solve  (scripts/solve_experiment.py)
# or NAME=FLAGS pairs, e.g.  scripts/build_exp.sh "P6W6=-DSFM_PPL32=6 -DSFM_SCORE_WAVES=6"
set -e
cd "$(dirname "$0")/../deep-sfm-revisited_amd/csrc"
mkdir -p ../../scripts/exp
build() {
  local name=$1; shift
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math -fno-slp-vectorize -fPIC -shared \
        -I../../include -Wno-unused-result "$@" -o ../../scripts/exp/libsfm_hip_$name.so \
        capi.hip ransac5.hip sweep.hip depth.hip irls.hip regularize.hip kinv.hip host_polish.cpp
}
if [ $# -eq 0 ]; then
  build STATS -DSFM_SCORE_STATS
  build SOLVESTATS -DSFM_SOLVE_STATS
else
  for spec in "$@"; do
    name=${spec%%=*}; flags=${spec#*=}
    # shellcheck disable=SC2086
    build "$name" $flags &
  done
  wait
fi
