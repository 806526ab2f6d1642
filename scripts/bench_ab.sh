#!/bin/bash
# Alternating bench A/B on one box: each argument set of SETS (separated by
# '|') runs ROUNDS times, interleaved; prints value / ms_per_step / the score
# and sweep launch times of every run.  Stops at the first failure.
#   SETS="--overlap-ref 0|--overlap-ref 1" ROUNDS=2 bash scripts/bench_ab.sh
set -u
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
IFS='|' read -r -a sets <<< "${SETS}"
for r in $(seq 1 ${ROUNDS:-2}); do
  for i in "${!sets[@]}"; do
    a=${sets[$i]}
    # shellcheck disable=SC2086
    timeout -k 10 300 python -u bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --no-regularize $a \
        > gpurun_out/ab_$i.log 2>&1 || { tail -20 gpurun_out/ab_$i.log; exit 1; }
    python - "$a" gpurun_out/ab_$i.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
k = d.get("kernel_ms", {})
rp = d.get("roofline_ref_planes") or {}
print(f"{sys.argv[1]:40s} {d['value']:9.1f} pairs/s  {d['ms_per_step']:.3f} ms/step  score {k.get('ransac_score', 0):.3f}"
      f"  sweep {k.get('plane_sweep', 0):.3f}  ref_planes {rp.get('avg_launch_ms', 0):.3f}  "
      f"sweep frac {d['roofline_sweep']['frac']}", flush=True)
PY
  done
done
