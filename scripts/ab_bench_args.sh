#!/bin/bash
# A/B bench lines with arbitrary bench.py arguments: each argument is one
# quoted argument string ("--config c4 --tune k=v"); lines go to
# gpurun_out/${TAG}_abx_<i>.log, the summary (value, scorer / sweep time and
# the sweep's HBM fraction) to stdout.
set -u
TAG=${TAG:-r05}
mkdir -p gpurun_out
i=0
for a in "$@"; do
  timeout -k 10 200 python -u bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --no-regularize $a \
      > gpurun_out/${TAG}_abx_$i.log 2>&1 || { tail -20 gpurun_out/${TAG}_abx_$i.log; exit 1; }
  python - gpurun_out/${TAG}_abx_$i.log "$a" <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][0]
k, sw = d["kernel_ms"], d["roofline_sweep"]
print(f"{sys.argv[2]:52s} {d['value']:9.1f} pairs/s  score {k.get('ransac_score', 0):.4f}  sweep {k.get('plane_sweep', 0):.4f}"
      f"  frac {sw['frac']:.4f}  GB {sw['bytes_per_launch'] / 1e9:.2f}", flush=True)
PY
  i=$((i+1))
done
