"""One bench step of a rocprofv3 --kernel-trace CSV: every kernel's start,
duration and the gap before it (usage: trace_step.py run_kernel_trace.csv)."""
import csv
import sys

NAMES = ["k_mf_cands", "k_score_mf2", "k_mf2_split", "k_mf2_lead", "k_mf2_keep", "k_select", "k_sweep_tile", "k_tgt_quads",
         "k_cand", "k_chain", "k_solve_back", "k_roots_split", "k_solve_front", "k_flow_points", "k_kinv3"]


def short(n):
    for k in NAMES:
        if k in n:
            return k
    return n[:30]


rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
seq = [(short(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
starts = [i for i, s in enumerate(seq) if s[0] == "k_kinv3"]
for j in range(len(starts) // 2, min(len(starts) // 2 + 2, len(starts) - 1)):
    i0, i1 = starts[j], starts[j + 1]
    t0, prev = seq[i0][1], None
    for n, a, b in seq[i0:i1]:
        if a - t0 > 2e7:
            break
        print(f"{n:16s} start {(a - t0) / 1e3:9.1f} us  dur {(b - a) / 1e3:8.1f} us  gap {(a - prev) / 1e3 if prev else 0:6.1f}")
        prev = b
    print()
