"""Summarise scripts/pmc_sweep.sh: mean per-dispatch SQ counters of the sweep
kernel (k_sweep*) per variant, and derived per-wave figures."""
import csv, glob, os
from collections import defaultdict
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
base = os.path.join(ROOT, "gpurun_out/pmcs")
names = dict(l.strip().split(": ", 1) for l in open(os.path.join(base, "variants.txt")) if ": " in l)
for v in sorted(names, key=lambda s: int(s[1:])):
    acc = defaultdict(list)
    dur = []
    for f in glob.glob(os.path.join(base, v, "**", "*counter_collection.csv"), recursive=True):
        per = defaultdict(float)
        for r in csv.DictReader(open(f)):
            if "k_sweep_rays" in r["Kernel_Name"] or "k_sweep" not in r["Kernel_Name"]:
                continue
            per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (d, c), val in per.items():
            acc[c].append(val)
    for f in glob.glob(os.path.join(base, v, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_sweep" in r["Kernel_Name"] and "k_sweep_rays" not in r["Kernel_Name"]:
                dur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
    m = {c: sum(x) / len(x) for c, x in acc.items() if x}
    ms = sorted(dur)[len(dur) // 2] if dur else float("nan")
    out = {"variant": names[v], "ms_median_profiled": round(ms, 3)}
    if "GRBM_GUI_ACTIVE" in m and dur:
        out["clock_ghz"] = round(m["GRBM_GUI_ACTIVE"] / 8 / (ms * 1e-3) / 1e9, 3)
    waves = m.get("SQ_WAVES")
    for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_WAVES"):
        if c in m:
            out[c] = "%.4g" % m[c]
            if waves and c != "SQ_WAVES":
                out[c + "/wave"] = round(m[c] / waves, 1)
    if "SQ_WAVE_CYCLES" in m:
        wc = m["SQ_WAVE_CYCLES"]
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
            if c in m:
                out[c + "/WAVE_CYC"] = round(m[c] / wc, 3)
        if waves:
            out["wave_cycles/wave(x4)"] = round(wc * 4 / waves, 0)
    if "SQ_INSTS_VALU" in m and dur and "clock_ghz" in out:
        cyc = ms * 1e-3 * out["clock_ghz"] * 1e9
        out["valu_issue_frac_2cyc"] = round(m["SQ_INSTS_VALU"] / 1024 * 2 / cyc, 3)
    print(out)
