#!/bin/bash
# A/B bench lines of library builds on one GPU box, alternating: each argument
# is a library path ("-" = the product libsfm_hip.so), optionally followed by
# "@key=v,key=v" (bench --tune), run ROUNDS (2) times in
# turn with the same bench arguments (BENCH_ARGS, default the c2 line without
# the CPU baseline).  Summary (value, scorer / sweep / solve ms) to stdout.
set -u
TAG=${TAG:-r06}
mkdir -p gpurun_out
i=0
for r in $(seq 1 ${ROUNDS:-2}); do
  for spec in "$@"; do
    lib=${spec%%@*}; tune=""; [ "$lib" != "$spec" ] && tune=${spec#*@}
    if [ "$lib" = "-" ]; then unset SFM_HIP_LIB; else export SFM_HIP_LIB=$lib; fi
    timeout -k 10 200 python -u bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --no-regularize \
        ${BENCH_ARGS:-} ${tune:+--tune $tune} > gpurun_out/${TAG}_abl_$i.log 2>&1 || { tail -20 gpurun_out/${TAG}_abl_$i.log; exit 1; }
    python - gpurun_out/${TAG}_abl_$i.log "$spec" <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][0]
k = d["kernel_ms"]
print(f"{sys.argv[2]:40s} {d['value']:9.1f} pairs/s  score {k.get('ransac_score', 0):.4f}  sweep {k.get('plane_sweep', 0):.4f}"
      f"  solve {k.get('ransac_solve', 0):.4f}", flush=True)
PY
    i=$((i+1))
  done
done
