#!/bin/bash
# A/B bench lines for tuning keys on one GPU box: each argument is one
# --tune string ("key=v,key=v"; "-" = defaults); CONFIG (c2) and STEPS (20)
# pick the workload.  Lines go to gpurun_out/${TAG}_ab_<i>.log and the
# summary (value, scorer time, sweep time, skipped share) to stdout.
set -u
TAG=${TAG:-r05}
CONFIG=${CONFIG:-c2}
mkdir -p gpurun_out
i=0
for t in "$@"; do
  tune=$t; [ "$t" = "-" ] && tune=""
  timeout -k 10 200 python -u bench.py --config $CONFIG --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline \
      --no-regularize ${tune:+--tune $tune} > gpurun_out/${TAG}_ab_$i.log 2>&1 || { tail -20 gpurun_out/${TAG}_ab_$i.log; exit 1; }
  python - gpurun_out/${TAG}_ab_$i.log "$t" <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][0]
r, k = d["roofline"], d["kernel_ms"]
w = r.get("work", "")
print(f"{sys.argv[2]:40s} {d['value']:9.1f} pairs/s  score {k.get('ransac_score', 0):.4f}  sweep {k.get('plane_sweep', 0):.4f}"
      f"  solve {k.get('ransac_solve', 0):.4f}  {w[w.rfind('('):] if '(' in w else ''}", flush=True)
PY
  i=$((i+1))
done
