"""Summarise scripts/pmc_kernel.sh: mean per-dispatch SQ counters of the
kernel matching argv[1], per variant, with per-wave and per-cycle ratios."""
import csv, glob, os, re, sys
from collections import defaultdict
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
base = os.path.join(ROOT, "gpurun_out/pmck")
rx = re.compile(sys.argv[1])
names = dict(l.strip().split(": ", 1) for l in open(os.path.join(base, "variants.txt")) if ": " in l)
for v in sorted(names, key=lambda s: int(s[1:])):
    acc = defaultdict(list)
    dur = []
    for f in glob.glob(os.path.join(base, v, "**", "*counter_collection.csv"), recursive=True):
        per = defaultdict(float)
        for r in csv.DictReader(open(f)):
            if rx.search(r["Kernel_Name"]):
                per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (d, c), val in per.items():
            acc[c].append(val)
    for f in glob.glob(os.path.join(base, v, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if rx.search(r["Kernel_Name"]):
                dur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
    m = {c: sum(x) / len(x) for c, x in acc.items() if x}
    ms = sorted(dur)[len(dur) // 2] if dur else float("nan")
    out = {"variant": names[v], "ms": round(ms, 3)}
    if "GRBM_GUI_ACTIVE" in m:
        out["ghz"] = round(m["GRBM_GUI_ACTIVE"] / 8 / (ms * 1e-3) / 1e9, 3)
    for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_WAVES"):
        if c in m:
            out[c] = "%.4g" % m[c]
    if "SQ_WAVE_CYCLES" in m:
        wc = m["SQ_WAVE_CYCLES"]
        for c in ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_SCA", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_INST_CYCLES_SALU"):
            if c in m:
                out[c + "/wave_cyc"] = round(m[c] / wc, 3)
    if "SQ_BUSY_CYCLES" in m and "SQ_VALU_MFMA_BUSY_CYCLES" in m:
        out["mfma_busy/busy"] = round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / m["SQ_BUSY_CYCLES"], 3)
    if "SQ_INSTS_VALU" in m and "ghz" in out:
        cyc = ms * 1e-3 * out["ghz"] * 1e9
        out["valu_issue_frac_2cyc"] = round(m["SQ_INSTS_VALU"] / 1024 * 2 / cyc, 3)
    if "SQ_INSTS_SALU" in m and "ghz" in out:
        cyc = ms * 1e-3 * out["ghz"] * 1e9
        out["salu_per_cu_cycle"] = round(m["SQ_INSTS_SALU"] / 256 / cyc, 3)
    print(out)
