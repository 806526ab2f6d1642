"""Per-kernel shader clock from a rocprofv3 --pmc GRBM_GUI_ACTIVE pass
(GRBM_GUI_ACTIVE / 8 XCDs / kernel duration).  Usage: pmc_clock.py DIR"""
import csv, glob, sys
from collections import defaultdict
d = sys.argv[1]
act = defaultdict(float)
dur = {}
name = {}
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
            act[r["Dispatch_Id"]] += float(r["Counter_Value"])
            name[r["Dispatch_Id"]] = r["Kernel_Name"][:40]
for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
rows = defaultdict(list)
for k, a in act.items():
    if k in dur and dur[k] > 0:
        rows[name[k]].append((dur[k] * 1e3, a / 8 / dur[k] / 1e9))
for n, v in rows.items():
    v = v[-4:]
    print(f"{n:40s} " + "  ".join(f"{ms:.3f} ms @ {ghz:.2f} GHz" for ms, ghz in v))
