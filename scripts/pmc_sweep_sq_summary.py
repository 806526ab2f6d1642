"""Summarise scripts/pmc_sweep_sq.sh output: per build, the mean per-dispatch
SQ counters of the sweep kernel and derived rates."""
import csv, glob, os, sys
from collections import defaultdict
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for name in sys.argv[1:]:
    acc = defaultdict(list)
    dur = []
    for f in glob.glob(os.path.join(ROOT, "gpurun_out/pmcs", name, "**", "*counter_collection.csv"), recursive=True):
        per = defaultdict(float)
        for r in csv.DictReader(open(f)):
            if "k_sweep" not in r["Kernel_Name"]:
                continue
            per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (d, c), v in per.items():
            acc[c].append(v)
    for f in glob.glob(os.path.join(ROOT, "gpurun_out/pmcs", name, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_sweep" in r["Kernel_Name"]:
                dur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
    m = {c: sum(v) / len(v) for c, v in acc.items() if v}
    ms = sorted(dur)[len(dur) // 2] if dur else float("nan")
    out = {"name": name, "ms_median": round(ms, 3)}
    if "GRBM_GUI_ACTIVE" in m and dur:
        out["clock_ghz"] = round(m["GRBM_GUI_ACTIVE"] / 8 / (ms * 1e-3) / 1e9, 3)
    for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAVES", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR"):
        if c in m:
            out[c] = "%.4g" % m[c]
    if "SQ_WAVE_CYCLES" in m:
        wc = m["SQ_WAVE_CYCLES"]
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
                  "SQ_INST_CYCLES_VMEM_WR"):
            if c in m:
                out[c + "/WAVE_CYC"] = round(m[c] / wc, 3)
        if "SQ_BUSY_CYCLES" in m and "SQ_ACTIVE_INST_VALU" in m:
            out["VALU_active/(BUSY*simds)"] = round(m["SQ_ACTIVE_INST_VALU"] / (m["SQ_BUSY_CYCLES"] * 4), 3)
    if "SQ_INSTS_VALU" in m and dur and "clock_ghz" in out:
        cyc = ms * 1e-3 * out["clock_ghz"] * 1e9
        out["valu_issue_frac_2cyc"] = round(m["SQ_INSTS_VALU"] / 1024 * 2 / cyc, 3)
    print(out)
