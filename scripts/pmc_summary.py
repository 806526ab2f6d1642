"""Summarise the rocprofv3 --pmc passes of scripts/gpu_pmc.sh into one JSON
per round (profiles/rNN_pmc.json): per-launch counters of the path's kernels.

HBM traffic follows /opt/skills/guides/MI355X_MICROARCH.md (HBM/rocprofv3):
FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the
bytes of wide coalesced reads, so it is doubled; WRITE_SIZE is taken as is
(calibrated for 16-byte-per-lane stores; for the sweep it matches the
algorithmic byte count of the volume to 0.2%).  Infinity-Cache hits are
counted in FETCH_SIZE, so re-reads of L3-resident inputs show up there.

usage: python scripts/pmc_summary.py gpurun_out/pmc profiles/r02_pmc_v1.json [config]
"""
import collections
import csv
import glob
import json
import os
import sys

KERNELS = {"k_sweep_flat": "plane_sweep", "k_score32": "ransac_score", "k_score": "ransac_score", "k_solve_front": "ransac_solve_front",
           "k_roots": "ransac_roots", "k_solve_back": "ransac_solve_back", "k_sweep": "plane_sweep", "k_solve": "ransac_solve",
           "k_chain": "ransac_chain", "k_cand": "ransac_chain", "k_tgt_quads": "sweep_tgt_quads", "k_flow_points": "flow_to_points"}


def short_name(name):
    """k_score_mf2 from a mangled or demangled kernel name."""
    import re
    m = re.match(r"_ZN\d+\w+?(\d+)(k_\w+)", name)
    if m:
        return m.group(2)[:int(m.group(1))]
    base = name.split("(")[0].split("<")[0]
    return base.split("::")[-1].split()[-1]


def kernel_key(name):
    if "k_score_mf" in name or "k_mf_cands" in name or "k_mf2_" in name:   # mangled names in the rocprof CSV
        return "ransac_score"
    if "k_sweep_tile" in name:
        return "plane_sweep"
    base = name.split("(")[0]
    for k, v in KERNELS.items():     # k_score32 is checked before k_score
        if base.endswith("::" + k) or ("::" + k + "<") in base:
            return v
    return None


# bench.py CONFIGS: (pairs per GPU, scene, iters, nlabel, cost dtype, keypoints)
WORKLOADS = {"c2": (8, 8, 128, "fp32"), "c3": (4, 8, 128, "bf16"), "c4": (8, 4, 64, "fp32"),
             "sparse": (8, 8, 128, "fp32"), "c5": (8, 16, 128, "fp32")}


def main(src, dst, config="c2"):
    # per (path key, kernel): one list of per-dispatch values per counter.  A
    # path key can hold several kernels of one step (ransac_score = k_mf_cands
    # + k_score_mf2 launches + k_mf2_split + k_mf2_lead + k_mf2_keep with pruning): its per-step
    # figure is the SUM of all their dispatches per step
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(os.path.join(src, "p*", "**", "*counter_collection.csv"), recursive=True)):
        acc = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            k = kernel_key(r["Kernel_Name"])
            if k:
                acc[(k, r["Kernel_Name"], r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (k, name, _, c), v in acc.items():
            per[(k, name)][c].append(v)
    keys = collections.defaultdict(list)
    for (k, name) in per:
        keys[k].append(name)
    out = {}
    for k, names in keys.items():
        m = collections.defaultdict(float)
        # per step: every dispatch of the key's kernels summed over the steps,
        # the step count being the fewest dispatches of any of them (k_mf_cands
        # once per step; the pruned scorer launches k_score_mf2 three times)
        steps = min(max(len(v) for v in per[(k, name)].values()) for name in names)
        for name in names:
            for c, v in per[(k, name)].items():
                m[c] += sum(v) / steps
        ls = collections.Counter()
        for n in names:                                  # template instances of one kernel add up
            ls[short_name(n)] += max(len(v) for v in per[(k, n)].values())
        d = {"launches_sampled": dict(ls)}
        d.update({c: round(v, 1) for c, v in sorted(m.items())})
        if "FETCH_SIZE" in m:
            d["hbm_read_bytes"] = int(m["FETCH_SIZE"] * 1024 * 2)
        if "WRITE_SIZE" in m:
            d["hbm_write_bytes"] = int(m["WRITE_SIZE"] * 1024)
        if "hbm_read_bytes" in d and "hbm_write_bytes" in d:
            d["hbm_bytes"] = d["hbm_read_bytes"] + d["hbm_write_bytes"]
        if "TCC_HIT_sum" in m:
            d["l2_hit_rate"] = round(m["TCC_HIT_sum"] / max(m["TCC_HIT_sum"] + m["TCC_MISS_sum"], 1), 4)
        if "SQ_INSTS_VALU" in m and "SQ_WAVES" in m:
            d["valu_insts_per_wave"] = round(m["SQ_INSTS_VALU"] / m["SQ_WAVES"], 1)
        if "SQ_ACTIVE_INST_VALU" in m and "SQ_WAVE_CYCLES" in m:
            d["valu_active_frac_of_wave_cycles"] = round(m["SQ_ACTIVE_INST_VALU"] / m["SQ_WAVE_CYCLES"], 4)
        out[k] = d
    b, it, nl, cd = WORKLOADS[config]
    json.dump({"source": "rocprofv3 --pmc --kernel-trace, separate passes (scripts/gpu_pmc.sh) over "
                         f"`python3 bench.py --config {config} --steps 1 --warmup 1 --no-cpu-baseline`",
               "workload": {"config": config, "batch": b, "nlabel": nl, "iters": it, "cost_dtype": cd},
               "src_hash": _src_hash(src),
               "kernels": out}, open(dst, "w"), indent=1, sort_keys=True)
    print(json.dumps({k: {x: v.get(x) for x in ("hbm_read_bytes", "hbm_write_bytes", "l2_hit_rate")}
                      for k, v in out.items()}, indent=1))


def _src_hash(src=None):
    """The src_hash of the profiled bench run (its JSON line in the pass logs
    of gpu_pmc.sh), else bench.src_hash() of the sources in this tree."""
    for log in sorted(glob.glob(os.path.join(src or "", "p*.log"))) if src else []:
        for line in open(log, errors="replace"):
            if line.startswith("{") and '"src_hash"' in line:
                try:
                    return json.loads(line)["src_hash"]
                except ValueError:
                    pass
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    return bench.src_hash()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], *(sys.argv[3:4]))
