#!/bin/bash
# Memory-pipeline counters (TA / TD / TCP) of the sweep kernel per variant
# (GPU box), kernel-trace only, one pass per block's counters.
# Usage: scripts/pmc_sweep_units.sh "k=v k=v" ...
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/pmcu
export TMPDIR=/tmp
n=0
: > gpurun_out/pmcu/variants.txt
for variant in "$@"; do
  n=$((n+1))
  i=0
  for set in "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE SQ_WAVES" \
             "TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE" \
             "TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum" \
             "TCP_TCR_TCP_STALL_CYCLES_sum TCP_TD_TCP_STALL_CYCLES_sum TCP_TOTAL_READ_sum TCP_TOTAL_WRITE_sum"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace --kernel-include-regex k_sweep \
        -d gpurun_out/pmcu/v$n/p$i -o run --output-format csv \
        -- python3 scripts/sweep_variant.py $variant > gpurun_out/pmcu/v$n.p$i.log 2>&1 \
        || { echo "pmc variant $n pass $i failed"; tail -5 gpurun_out/pmcu/v$n.p$i.log; exit 1; }
  done
  echo "v$n: $variant" >> gpurun_out/pmcu/variants.txt
done
python3 - <<'PY'
import csv, glob, collections
names = dict(l.strip().split(": ", 1) for l in open("gpurun_out/pmcu/variants.txt") if ": " in l)
for v in sorted(names, key=lambda s: int(s[1:])):
    acc = collections.defaultdict(list)
    for f in glob.glob(f"gpurun_out/pmcu/{v}/**/*counter_collection.csv", recursive=True):
        per = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (d, c), x in per.items():
            acc[c].append(x)
    m = {c: sum(x) / len(x) for c, x in acc.items()}
    g = m.get("GRBM_GUI_ACTIVE", 1.0)
    print(names[v], {c: round(x / g, 3) if c != "GRBM_GUI_ACTIVE" else x for c, x in sorted(m.items())})
PY
