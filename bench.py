#!/usr/bin/env python3
"""Benchmark: image-pairs/sec of the two-view SfM hot path on MI355X.

One step = one batch of `--batch` pairs per GPU through
    flow -> correspondences -> RANSAC five-point (H = 512 x iters)
    -> pose (RESCALE_DEPTH, NORM_TARGET 0.6) -> plane-sweep cost volume
with every input already resident in HBM.  ``--pipeline`` overlaps
consecutive steps (each step's sweep on a side stream beside the next step's
pose stage); the timed region ends after the last sweep either way.
``--config`` picks the workload
(BASELINE.json configs):

  c2      (default) 8 KITTI 376x1242 pairs, dense flow N=435,032, H=4096,
          L=128, fp32 volume [8, 64, 128, 94, 311]        (configs[1])
  c3      4 KITTI pairs per GPU, bf16 volume: the 8-GPU data-parallel shape
          (32 pairs on 8 GPUs)                              (configs[2])
  c4      8 indoor 640x480 pairs, N=285,200, H=2048, L=64 (configs[3])
  sparse  c2 with the SIFT-keypoint branch of pose_by_ransac: N=2,048
          keypoints per pair (SFMnet.py:250-254); the solve dominates
  c5      c2 with H=8192 hypotheses (ransac_iter 16; LO-RANSAC's count,
          configs[4]; its IRLS refinement is not in the step)

Multi-GPU: one process per GPU.  Under torchrun the ranks come from its env;
``python bench.py --gpus N`` with no WORLD_SIZE starts the N ranks itself
(fresh child processes, before anything touches the GPU).  Pairs shard
across ranks with no data-path collective ("scaling": "weak"); RCCL only for
the barrier, the max-over-ranks timing reduction and the device-name gather.

Rank 0 prints ONE JSON line.  `roofline` is the dominant kernel (RANSAC
scoring: k_score_mf on the f16 matrix cores, or k_score32 on the fp32 VALU
when the matrix-core scorer is off); `roofline_sweep` the HBM-bound
cost-volume kernel; both
average launch durations come from HIP events recorded by libsfm_hip around
every launch on the launching stream during the timed region; `traffic` is
the PMC-measured HBM bytes per launch (FETCH_SIZE x2 + WRITE_SIZE, gfx950
correction) from the committed profiles/rNN_pmc*.json of the same workload.
The `cpu_baseline` is the oracle (CPU restatement) on one full pair, rank 0 at
N=1 only.
"""
import argparse
import json
import os
import re
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "deep-sfm-revisited_amd"))

PEAK_HBM_GBS = 8000.0        # MI355X HBM3E spec (MI355X_MICROARCH.md)
PEAK_FP64_TFLOPS = 78.6      # MI355X fp64 vector spec
PEAK_FP32_TFLOPS = 157.3     # MI355X fp32 vector spec (MI355X_MICROARCH.md)
PEAK_BF16_TFLOPS = 2500.0    # MI355X dense bf16 MFMA (MI355X_MICROARCH.md; no sparsity)
PEAK_F16_TFLOPS = 2500.0     # MI355X dense f16 MFMA (same rate as bf16; no sparsity)
PEAK_F32_MFMA_TFLOPS = 157.3 # MI355X f32 MFMA (v_mfma_f32_32x32x2_f32 = the f32 vector rate; MI355X_MICROARCH.md)
FLOP_PER_EVAL = 50           # Ex, xE, x'Ex, sqrt, div, |.|
MF_MFMA_FLOP_PER_EVAL = 128  # k_score_mf: 4 x v_mfma_f32_32x32x16_f16 (32768 FLOP each) per 32x32 evaluations

# name -> (pairs per GPU, image hw, ransac_iter, nlabel, cost dtype, sparse keypoints per pair)
CONFIGS = {
    "c2": (8, "kitti", 8, 128, "fp32", 0),
    "c3": (4, "kitti", 8, 128, "bf16", 0),
    "c4": (8, "indoor", 4, 64, "fp32", 0),
    "sparse": (8, "kitti", 8, 128, "fp32", 2048),
    "c5": (8, "kitti", 16, 128, "fp32", 0),      # H = 8192 hypotheses (LO-RANSAC's count; its IRLS is not timed)
}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", choices=sorted(CONFIGS), default="c2")
    ap.add_argument("--batch", type=int, default=None, help="pairs per GPU per step (default: the config's)")
    ap.add_argument("--nlabel", type=int, default=None)
    ap.add_argument("--iters", type=int, default=None, help="ransac_iter (H = 512 x iters)")
    ap.add_argument("--threshold", type=float, default=1e-4)
    ap.add_argument("--cost-dtype", choices=["fp32", "bf16"], default=None)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-regularize", action="store_true",
                    help="skip the (unscored) PSNet 3-D regularisation roofline line after the timed region")
    ap.add_argument("--fused", action="store_true",
                    help="(the default for dense flow since round 6) RANSAC reads the flow directly "
                         "(sfm_ransac5_flow, SURVEY 8f row 2) instead of materialised correspondences")
    ap.add_argument("--no-fused", action="store_true",
                    help="materialise the correspondences first (sfm_flow_to_points + sfm_ransac5_packed): "
                         "0.6 - 1.5 %% slower at c2, profiles/r06_fused_ab.txt")
    ap.add_argument("--cpu-threads", type=int, default=16,
                    help="host threads for the CPU baseline: 16 = the host-core share one GPU gets on the "
                         "MI355X pool (nproc there reports the whole 256-thread host)")
    ap.add_argument("--cpu-runs", type=int, default=5, help="full-pair CPU baseline runs (median; BASELINE.md: >= 5)")
    ap.add_argument("--pipeline", action="store_true",
                    help="each step's sweep on a side stream, overlapping the next step's pose stage, the "
                         "next scorer held for it (TwoViewHotPath.step_pipelined, sfm_score_gate): round 5 c2 "
                         "+0.2 %%, c4 / sparse +5 %%, c3 +0.6 %% pairs/s (profiles/r05_pipeline_gate_ab.txt); the "
                         "overlapped kernels' launch durations (the roofline fields) then include the overlap")
    ap.add_argument("--no-gate", action="store_true",
                    help="with --pipeline: do not hold the next step's scorer for the side-stream sweep "
                         "(sfm_score_gate); the sweep then overlaps the scorer too")
    ap.add_argument("--overlap-ref", default="0", choices=("0", "score", "step"),
                    help="the cost volume's pose-independent reference half on a side stream "
                         "(TwoViewHotPath.step_overlap): 'score' beside the RANSAC scorer (behind the score fence), "
                         "'step' from the start of the step; the sweep after RANSAC then writes the warped half")
    ap.add_argument("--tune", default="",
                    help="launch-shape tuning keys for A/B runs, 'key=value,key=value' (sfm_tune_set; "
                         "include/sfm_hip.h lists them); recorded in config.tune")
    args = ap.parse_args(argv)
    if args.pipeline and args.overlap_ref != "0":
        # step_pipelined writes the whole volume and ignores overlap_ref: the
        # warped-half byte count would misstate the sweep's traffic
        ap.error("--pipeline and --overlap-ref are exclusive")
    b, hw, it, nl, cd, kp = CONFIGS[args.config]
    args.batch = b if args.batch is None else args.batch
    args.iters = it if args.iters is None else args.iters
    args.nlabel = nl if args.nlabel is None else args.nlabel
    args.cost_dtype = cd if args.cost_dtype is None else args.cost_dtype
    args.hw_name = hw
    args.keypoints = kp
    return args


def src_hash():
    """Hash of the kernel and C-ABI sources (comments and whitespace removed,
    so documentation edits keep it): ties a committed rocprofv3 / PMC summary
    to the code it was recorded from."""
    import hashlib
    h = hashlib.sha256()
    csrc = os.path.join(ROOT, "deep-sfm-revisited_amd", "csrc")
    files = sorted(f for f in os.listdir(csrc) if f.endswith((".hip", ".h", ".cpp")))
    for f in [os.path.join(csrc, f) for f in files] + [os.path.join(ROOT, "include", "sfm_hip.h")]:
        t = open(f).read()
        t = re.sub(r"/\*.*?\*/", " ", t, flags=re.S)
        t = re.sub(r"//[^\n]*", " ", t)
        h.update(os.path.basename(f).encode() + b"\0" + " ".join(t.split()).encode() + b"\0")
    return h.hexdigest()[:16]


def _profile_hash(path):
    """src_hash a committed summary was recorded with: a PMC summary's own
    "src_hash" field, or a stats CSV's sidecar <name>.meta.json."""
    try:
        if path.endswith(".json"):
            return json.load(open(path)).get("src_hash")
        return json.load(open(path[:-4] + ".meta.json")).get("src_hash")
    except (OSError, ValueError):
        return None


def _round_version(path):
    """profiles/r02_pmc_v10.json -> (2, 10): numeric, so v10 sorts after v6
    (an optional config tag, r02_pmc_c3_v1.json, is allowed)."""
    m = re.search(r"r(\d+)_pmc(?:_(?!v\d)[a-z0-9]+)?(?:_v(\d+))?\.json$", os.path.basename(path))
    return (int(m.group(1)), int(m.group(2) or 0)) if m else (-1, -1)


def pmc_traffic(args):
    """HBM bytes per launch of the path's kernels from the newest committed PMC
    summary (profiles/rNN_pmc[_vK].json, scripts/gpu_pmc.sh + scripts/pmc_summary.py;
    counters need their own profiler pass, so they cannot be read live here).
    Only reported for the workload the summary was collected on, and only from
    a summary recorded from these sources (src_hash)."""
    import glob
    cur = src_hash()
    fs = [f for f in glob.glob(os.path.join(ROOT, "profiles", "r*_pmc*.json"))
          if _round_version(f)[0] >= 0 and _profile_hash(f) == cur]
    fs.sort(key=_round_version)
    for f in reversed(fs):
        d = json.load(open(f))
        wl = d.get("workload", {"config": "c2", "batch": 8, "nlabel": 128, "iters": 8, "cost_dtype": "fp32"})
        if (wl.get("config", "c2"), wl.get("batch"), wl.get("nlabel"), wl.get("iters"), wl.get("cost_dtype")) == \
                (args.config, args.batch, args.nlabel, args.iters, args.cost_dtype):
            return {n: v.get("hbm_bytes") for n, v in d["kernels"].items()}, os.path.relpath(f, ROOT)
    return {}, None


def pmc_kernel_counters(traffic_src, region):
    """The raw counters of one region of the PMC summary ``pmc_traffic``
    matched (same workload, same sources), or None."""
    if not traffic_src:
        return None
    try:
        return json.load(open(os.path.join(ROOT, traffic_src)))["kernels"].get(region)
    except (OSError, ValueError, KeyError):
        return None


VALU_ISSUE_CYCLES = 4       # MI355X_MICROARCH.md: vector-instruction issue cost per instruction (one wave's stream)
N_SIMD, N_XCD = 1024, 8     # 256 CUs x 4 SIMDs in 8 XCDs


def valu_issue(counters):
    """What bounds k_score_mf2: VALU instructions x the
    guide's issue cost against the SIMDs' cycles over the launch, from the
    PMC summary's SQ_INSTS_VALU and GRBM_GUI_ACTIVE (GPU-busy cycles summed
    over the 8 XCDs; per launch).  1.0 = every SIMD issuing a VALU
    instruction every VALU_ISSUE_CYCLES for the whole launch."""
    if not counters or not counters.get("SQ_INSTS_VALU") or not counters.get("GRBM_GUI_ACTIVE"):
        return None
    cycles = counters["GRBM_GUI_ACTIVE"] / N_XCD
    insts = counters["SQ_INSTS_VALU"]
    return {"insts_per_launch": int(insts), "issue_cycles_per_inst": VALU_ISSUE_CYCLES,
            "simd_cycles_per_launch": int(cycles), "frac": round(insts * VALU_ISSUE_CYCLES / (N_SIMD * cycles), 4),
            "note": "VALU issue utilisation from the PMC summary (profiled run; SQ_INSTS_VALU includes the MFMAs)"}


def _stats_version(path):
    """profiles/r03_kernel_stats_v4.csv -> (3, 4); a config tag (r03_kernel_stats_c3_v1.csv) is allowed."""
    m = re.search(r"r(\d+)_kernel_stats(?:_(?!v\d)([a-z0-9]+))?(?:_v(\d+))?\.csv$", os.path.basename(path))
    if not m:
        return None
    tag = m.group(2) or "c2"
    return tag, (int(m.group(1)), int(m.group(3) or 0))


def rocprof_kernel_ms(args, prefixes, optional=()):
    """Time per step (ms) of the kernels named by ``prefixes`` (+ ``optional``
    ones when present) from the newest committed rocprofv3 --stats summary of
    this workload (profiles/rNN_kernel_stats[_cfg]_vK.csv, written by
    scripts/gpu_evidence.sh from a profiled run of this bench): their total
    durations summed over the calls of the first prefix (one launch per step;
    the pruned scorer launches k_score_mf2 twice per step), so the line
    carries a frac that follows from the committed profile, beside the live
    HIP-event one.  Only a summary recorded from these sources counts (its
    .meta.json sidecar's src_hash)."""
    import csv
    import glob
    best = None
    cur = src_hash()
    for f in glob.glob(os.path.join(ROOT, "profiles", "r*_kernel_stats*.csv")):
        v = _stats_version(f)
        if v and v[0] == args.config and _profile_hash(f) == cur and (best is None or v[1] > best[0]):
            best = (v[1], f)
    if best is None:
        return None, None
    tot, hit, calls = 0.0, set(), {}
    with open(best[1]) as fh:
        for row in csv.DictReader(fh):
            for p in tuple(prefixes) + tuple(optional):
                # whole kernel names: mangled (length-prefixed, "11k_score_mf2") or demangled
                if f"{len(p)}{p}" in row["Name"] or re.search(r"\b" + re.escape(p) + r"[<(]", row["Name"]):
                    tot += float(row["TotalDurationNs"]) * 1e-6
                    calls[p] = calls.get(p, 0) + int(row["Calls"])
                    hit.add(p)
                    break
    # every named kernel must be in the summary (an older scorer's profile does not count)
    if not set(prefixes) <= hit or not calls.get(prefixes[0]):
        return None, os.path.relpath(best[1], ROOT)
    return tot / calls[prefixes[0]], os.path.relpath(best[1], ROOT)


ROOFLINE_REGIONS = ("ransac_score", "plane_sweep", "ref_planes")
ALL_REGIONS = ("flow_to_points", "keypoints_to_points", "ransac_solve", "ransac_chain", "ransac_score",
               "ransac_select", "plane_sweep", "ref_planes")


def profiled_pass(stepf, inputs, steps, dev):
    """Average launch time of every profiled stage over `steps` extra steps
    with all regions evented (outside the timed region)."""
    import torch
    from sfm_amd import _lib
    torch.cuda.synchronize(dev)
    _lib.profile_reset()
    _lib.profile_select(None)
    _lib.profile_enable(True)
    for _ in range(steps):
        stepf(*inputs)
    torch.cuda.synchronize(dev)
    _lib.profile_enable(False)
    kt = {}
    for name in ALL_REGIONS:
        ms, n = _lib.profile_read(name)
        if n:
            kt[name] = ms / n
    return kt


def score_roofline(use_mf, tflops, done, evals, skipped, cands, n, ms, traffic, traffic_src, rocprof=None,
                   scorer=None, upper=None):
    """Roofline line of the RANSAC scoring kernel.  achieved = the algorithmic
    rate (50 FLOP per (candidate E, correspondence) evaluation);
    peak = the unit that executes it: the dense f16 MFMA peak for k_score_mf
    (exact decisions from split-f16 matrix-core products, csrc/score_mf.h), the
    fp32 VALU peak for k_score32.  For k_score_mf `mfma_issued` is the MFMA
    pipe's own utilisation (4 MFMAs per 1024 evaluations): the kernel's floor."""
    work = (f"{done} evals x {FLOP_PER_EVAL} FLOP per launch: {cands} candidate E x N={n} = {evals}, "
            f"minus {skipped} skipped by exact count-bound pruning ({100.0 * skipped / max(evals, 1):.1f}%)")
    issued_flop = done * MF_MFMA_FLOP_PER_EVAL
    if upper is not None:
        # the one-sided pruning (score_mf_prune_upper): every candidate's
        # evaluations before the pruning point take the one-sided test (3 MFMAs
        # per 32x32), the kept candidates are rescored two-sided over every point
        one, two, kept = upper
        issued_flop = one * MF_MFMA_FLOP_PER_EVAL * 3 // 4 + two * MF_MFMA_FLOP_PER_EVAL
        work += (f"; one-sided pass (points not certainly outliers, upper-bound counts): {one} evals; "
                 f"{kept} of {cands} candidates kept and counted exactly over every point (float64, or two-sided past 256 per pair): {two} evals")
    if use_mf:
        issued = issued_flop / (ms * 1e-3) / 1e12
        rp = None
        if rocprof and rocprof[0]:
            t = done * FLOP_PER_EVAL / (rocprof[0] * 1e-3) / 1e12
            rp = {"avg_launch_ms": round(rocprof[0], 4), "achieved": round(t, 3),
                  "frac": round(t / PEAK_F16_TFLOPS, 4), "source": rocprof[1],
                  "note": "k_mf_cands + k_score_mf2 (+ k_mf2_split + k_mf2_lead + k_mf2_keep + k_mf2_keep_map + "
                          "k_mf2_zero_kept + k_mf2_exact) per step from the committed rocprofv3 --stats "
                          "summary of this workload (a profiled run clocks lower than this one)"}
        pruned = scorer == "k_score_mf2+prune"
        kern = ("ransac_score (k_mf_cands + k_score_mf2 x3 + k_mf2_split + k_mf2_lead + k_mf2_keep: count-bound pruning)" if pruned
                else "ransac_score (k_mf_cands + k_score_mf2)")
        if pruned and upper is not None:
            kern = ("ransac_score (k_mf_cands + k_score_mf2 one-sided x3 + k_mf2_split + k_mf2_lead + k_mf2_keep + "
                    "k_mf2_keep_map + k_mf2_zero_kept + k_mf2_exact + k_score_mf2 two-sided: one-sided count-bound "
                    "pruning)")
        return {"kernel": kern, "scorer": scorer, "bound": "mfma-f16", "achieved": round(tflops, 3),
                "peak": PEAK_F16_TFLOPS, "unit": "TFLOP/s", "frac": round(tflops / PEAK_F16_TFLOPS, 4),
                "mfma_issued": {"flop_per_eval": MF_MFMA_FLOP_PER_EVAL if upper is None else "96 one-sided, 128 two-sided",
                                "tflops": round(issued, 1),
                                "frac": round(issued / PEAK_F16_TFLOPS, 4)},
                "traffic": traffic, "traffic_source": traffic_src, "avg_launch_ms": round(ms, 4), "work": work,
                "rocprof": rp, "valu_issue": valu_issue(pmc_kernel_counters(traffic_src, "ransac_score"))}
    return {"kernel": "ransac_score (k_score32)", "bound": "valu-fp32", "achieved": round(tflops, 3),
            "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s", "frac": round(tflops / PEAK_FP32_TFLOPS, 4),
            "traffic": traffic, "traffic_source": traffic_src, "avg_launch_ms": round(ms, 4), "work": work}


def metric_name(nlabel, hwtxt):
    """BASELINE.json's metric for its own workload (KITTI, nlabel=128); the
    same form with this run's plane count and image shape otherwise."""
    if nlabel == 128 and hwtxt.startswith("KITTI"):
        return "image-pairs/sec (5-pt RANSAC + nlabel=128 plane-sweep), KITTI 376\u00d71242"
    return f"image-pairs/sec (5-pt RANSAC + nlabel={nlabel} plane-sweep), {hwtxt}"


def cpu_info(threads):
    import torch
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"cores": threads, "nproc": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)),
            "torch_threads": torch.get_num_threads(), "cpu_model": model}


def cpu_baseline(flow, K, ref_fea, tgt_fea, pose, args, n_pts=None, keypoints=None):
    """Oracle (CPU restatement) on one full pair of the same workload: RANSAC
    with all 512 chains x `iters` on all N correspondences (C++, OpenMP over
    chains) and the full L-plane sweep (torch-CPU fp32), after a warm-up; the
    median of ``--cpu-runs`` runs."""
    import numpy as np
    import torch
    sys.path.insert(0, ROOT)
    from oracle import ransac5 as ORR
    from oracle import sweep as OSW
    from sfm_amd import ransac
    threads = max(1, min(args.cpu_threads, len(os.sched_getaffinity(0))))
    torch.set_num_threads(threads)
    Kinv = torch.inverse(K[:1].cpu())
    if keypoints is None:
        pts = ransac.flow_to_points(flow[:1], Kinv.to(flow.device)).cpu().numpy()[0]
    else:
        pts = ransac.gather_keypoints(flow[:1], Kinv.to(flow.device), keypoints[:1], [n_pts]).cpu().numpy()[0]
    q, qp = np.ascontiguousarray(pts[:, :2]), np.ascontiguousarray(pts[:, 2:])
    r = ref_fea[:1].cpu().float(); t = tgt_fea[:1].cpu().float(); P = pose[:1].cpu(); Kc = K[:1].cpu()
    ORR.ransac5(q[:2000], qp[:2000], iters=1, thr=args.threshold, nchains=8, nthreads=threads)   # warm-up
    OSW.plane_sweep_cost(r, t, P, Kc, torch.inverse(Kc), args.nlabel, 1.0, rescale=0.6, planes=[0, 1])
    tr, ts = [], []
    for _ in range(max(1, args.cpu_runs)):
        t0 = time.perf_counter()
        ORR.ransac5(q, qp, iters=args.iters, thr=args.threshold, nchains=512, nthreads=threads)
        tr.append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        OSW.plane_sweep_cost(r, t, P, Kc, torch.inverse(Kc), args.nlabel, 1.0, rescale=0.6)
        ts.append(time.perf_counter() - t0)
    t_ransac = float(np.median(tr))
    t_sweep = float(np.median(ts))
    per_pair = t_ransac + t_sweep
    out = {"value": round(1.0 / per_pair, 4), "unit": "pairs/s", "kind": "port",
           "sample": (f"1 full pair, median of {len(tr)} runs after a warm-up: RANSAC 512 chains x {args.iters} "
                      f"iters on N={q.shape[0]} ({t_ransac:.2f} s, oracle C++ OpenMP), {args.nlabel}-plane sweep "
                      f"({t_sweep:.3f} s, torch-CPU fp32)"),
           "runs_s": [round(a + b, 3) for a, b in zip(tr, ts)]}
    out.update(cpu_info(threads))
    out["threads_reason"] = ("the host-core share of one GPU on this pool (16); nproc/affinity show the whole "
                             "host" if threads == 16 else "--cpu-threads")
    return out


def regularize_roofline(cost, steps=3, precision="bf16"):
    """PSNet's 12-layer 3-D cost regularisation on the first pair of the last
    step's cost volume, after the timed region: sfm_conv3_bf16 (bf16 MFMA,
    the fast option), sfm_conv3_f16 (precision "fp16": f16 MFMA, the
    reference's precision under cfg.MIXED_PREC) or sfm_conv3_f32 (precision
    "fp32": f32 MFMA, the reference's precision).  Not part of ``value`` (the metric's path ends at
    the cost volume); reported so the MFMA kernels' rooflines are measured
    live beside the path's."""
    import torch
    from sfm_amd import _lib
    from sfm_amd.regularize import CostRegularization
    torch.manual_seed(0)
    reg = CostRegularization(cost.shape[1]).to(cost.device).eval()
    one = cost[:1]
    reg(one, precision=precision)
    torch.cuda.synchronize(cost.device)
    _lib.profile_reset()
    _lib.profile_enable(True)
    for _ in range(steps):
        reg(one, precision=precision)
    torch.cuda.synchronize(cost.device)
    _lib.profile_enable(False)
    ms, n = _lib.profile_read({"bf16": "conv3", "fp16": "conv3_f16", "fp32": "conv3_f32",
                               "fp32x3": "conv3_f32x3"}[precision])
    _, L, h, w = one.shape[1:]
    vox = L * h * w
    flop = 2 * vox * 27 * (one.shape[1] * 32 + 10 * 32 * 32 + 32)
    per_stack = ms / steps
    tf = flop / (per_stack * 1e-3) / 1e12
    peak = PEAK_F32_MFMA_TFLOPS if precision == "fp32" else PEAK_BF16_TFLOPS   # f16 dense = bf16 dense
    if precision == "fp32x3":
        # algorithmic fp32 FLOP against the f16 dense peak: the matrix cores
        # issue 3x that (three split products per fp32 product)
        return {"kernel": "conv3 x12 (PSNet dres0..classify, fp32 products from 3 split-f16 MFMAs)",
                "bound": "mfma-f16", "achieved": round(tf, 1), "peak": peak, "unit": "TFLOP/s",
                "frac": round(tf / peak, 4), "mfma_issued_frac": round(3 * tf / peak, 4),
                "avg_launch_ms": round(ms / max(n, 1), 4), "ms_per_stack": round(per_stack, 4),
                "work": f"{flop} FLOP per stack (1 pair, L={L}, {h}x{w}; 2*27*Cin*Cout per voxel and layer)",
                "note": "not part of value: the CNN after the measured path, timed after it"}
    return {"kernel": f"conv3 x12 (PSNet dres0..classify, {precision} MFMA)", "bound": f"mfma-{precision}",
            "achieved": round(tf, 1), "peak": peak, "unit": "TFLOP/s", "frac": round(tf / peak, 4),
            "avg_launch_ms": round(ms / max(n, 1), 4), "ms_per_stack": round(per_stack, 4),
            "work": f"{flop} FLOP per stack (1 pair, L={L}, {h}x{w}; 2*27*Cin*Cout per voxel and layer)",
            "note": "not part of value: the CNN after the measured path, timed after it"}


def rank_device_index(local):
    """The GPU a rank drives: its LOCAL_RANK (one process per GPU of the node;
    dist.init binds the RCCL communicator to the same index).  Under
    SFM_BENCH_SHARED_GPU=1 (a rehearsal of the N-rank path on a one-GPU box,
    never a measurement) every rank drives device 0."""
    return 0 if _shared_gpu() else int(local)


def _shared_gpu():
    """SFM_BENCH_SHARED_GPU=1: every rank on device 0 over gloo -- the real
    GPU step, rank sharding, barrier, max-over-ranks timing and gather run
    with N ranks on a one-GPU box (tests/test_gpu_bench_ranks.py).  The line
    is marked "rehearsal" and its value is not a multi-GPU measurement."""
    return os.environ.get("SFM_BENCH_SHARED_GPU") == "1"


def _stub_mode():
    """SFM_BENCH_CPU_STUB=1: CPU-only rehearsal of the launch / rank / timing
    control flow (gloo, a small torch matmul as the step).  Used by
    tests/test_bench_launch.py; never a measurement."""
    return os.environ.get("SFM_BENCH_CPU_STUB") == "1"


def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    args = parse(argv)
    if args.gpus < 1:
        print("bench: --gpus must be >= 1", file=sys.stderr)
        return 2
    from sfm_amd import dist     # torch only: nothing here touches the GPU
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # no torchrun: start the N ranks as fresh children and pass on their exit code
        return dist.launch_local(args.gpus, [sys.executable, os.path.abspath(__file__)] + argv)
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if world_env != args.gpus:
        print(f"bench: --gpus {args.gpus} but WORLD_SIZE={world_env}: refusing to report a "
              f"{world_env}-rank run as {args.gpus}", file=sys.stderr)
        return 2
    if _stub_mode():
        return _main_stub(args, dist)
    return _main_gpu(args, dist)


def _main_stub(args, dist):
    import torch
    rank, world, _local = dist.init(backend="gloo")
    x = torch.randn(64, 64, generator=torch.Generator().manual_seed(rank))
    for _ in range(args.warmup):
        x = torch.tanh(x @ x)
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        x = torch.tanh(x @ x)
    dist.barrier()
    elapsed = dist.reduce_max(time.perf_counter() - t0)
    names = dist.device_names(None)
    # the same per-pair gather as the GPU path: rows tagged (rank, device index, pair)
    di = rank_device_index(_local)
    rows = torch.tensor([[float(rank), float(di), float(i)] for i in range(args.batch)], dtype=torch.float64)
    gathered = dist.gather_rows(rows, world)
    if rank == 0:
        print(json.dumps({"metric": "stub", "value": world * args.batch * args.steps / elapsed, "unit": "pairs/s",
                          "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "gathered": {"pairs": int(gathered.shape[0]), "rows": gathered.tolist()},
                          "dist": {"world_size": torch.distributed.get_world_size() if torch.distributed.is_initialized() else 1,
                                   "backend": torch.distributed.get_backend() if torch.distributed.is_initialized() else None,
                                   "devices": names},
                          "config": {"name": args.config, "pairs_per_gpu": args.batch,
                                     "global_batch": world * args.batch}}), flush=True)
    if torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()
    return 0


def _main_gpu(args, dist):
    import torch
    from sfm_amd import _lib, ransac, synth
    from sfm_amd.pipeline import TwoViewHotPath
    rank, world, local = dist.init(backend="gloo" if _shared_gpu() else None)
    dev = torch.device("cuda", rank_device_index(local))
    torch.cuda.set_device(dev)
    B = args.batch
    if args.hw_name == "kitti":
        hw, kcal, hwtxt = synth.KITTI_HW, None, "KITTI 376x1242"
    else:
        hw, kcal, hwtxt = synth.INDOOR_HW, synth.INDOOR_K, "indoor 640x480"
    fhw = synth.feature_hw(hw)
    C = 32
    cost_dtype = torch.float32 if args.cost_dtype == "fp32" else torch.bfloat16

    # synthetic inputs, distinct pairs per rank, resident in HBM before timing
    flow, K, pose_gt, _ = synth.kitti_pair_batch(B, seed=1000 + rank, hw=hw, device=dev, k=kcal)
    ref_fea, tgt_fea = synth.features(B, C, fhw[0], fhw[1], seed=rank, device=dev)
    kp = None
    if args.keypoints:
        kp = synth.keypoints(B, args.keypoints, hw, seed=rank, device=dev)
    for kv in filter(None, args.tune.split(",")):
        k, v = kv.split("=")
        _lib.tune(k.strip(), int(v))
    hp = TwoViewHotPath(B, hw, fhw, C, args.nlabel, args.iters, args.threshold, 1.0, rescale_depth=True,
                        norm_target=0.6, cost_dtype=cost_dtype, device=dev,
                        fused=not args.keypoints and not args.no_fused,
                        keypoints=None if kp is None else (kp, [args.keypoints] * B),
                        overlap_ref=False if args.overlap_ref == "0" else args.overlap_ref,
                        gate_scorer=not args.no_gate)

    # --pipeline: step i's sweep (side stream) overlaps step i+1's pose stage
    stepf = hp.step_pipelined if args.pipeline else hp.step
    for _ in range(args.warmup):
        stepf(flow, K, ref_fea, tgt_fea)
    torch.cuda.synchronize(dev)
    # HIP events inside the timed region only around the two roofline kernels:
    # every evented launch adds two event records to the stream (sparse step
    # 1.722 -> 1.772 ms with all seven regions evented, git-history scripts/event_ab.py)
    _lib.profile_reset()
    _lib.profile_select(ROOFLINE_REGIONS)
    _lib.profile_enable(True)
    dist.barrier(dev)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        E, P, inl, cost = stepf(flow, K, ref_fea, tgt_fea)
    torch.cuda.synchronize(dev)
    dist.barrier(dev)
    elapsed = time.perf_counter() - t0
    _lib.profile_enable(False)
    elapsed = dist.reduce_max(elapsed, dev)
    names = dist.device_names(dev)
    # validation outputs of every rank's pairs to rank 0 (replaces
    # DataParallel's output gather, main.py:219): E[9], P[12], inliers per pair
    rows = torch.cat([E.reshape(B, 9), P.reshape(B, 12), inl.reshape(B, 1).double()], 1)
    gathered = dist.gather_rows(rows, world).cpu()

    kt = {}
    for name in ROOFLINE_REGIONS:
        ms, n = _lib.profile_read(name)
        if n:
            kt[name] = ms / n
    # the other stages' launch times: a separate, fully evented pass after the
    # timed region (same inputs and outputs; never part of `value`)
    kt_all = profiled_pass(stepf, (flow, K, ref_fea, tgt_fea), min(args.steps, 5), dev)
    cands = ransac.candidate_counts(hp.ws, B, args.iters)
    evals = sum(cands) * hp.n                       # candidate E x correspondences per launch
    skipped = ransac.skipped_evaluations(hp.ws, B, args.iters)   # exact bound pruning (last launch)
    done = evals - skipped                          # evaluations the launch performed
    upper_work = None
    if _lib.last_scorer() == "k_score_mf2+prune" and _lib.tune_get("score_mf_prune_upper"):
        # every evaluation not skipped took the one-sided test (all candidates
        # before the pruning point, the first keep's survivors after it); the
        # finally kept candidates were then counted exactly over every point
        kept = ransac.kept_candidates(hp.ws, B, args.iters)
        upper_work = (done, int(kept.sum()) * hp.n, int(kept.sum()))
    score_ms = kt["ransac_score"]
    score_tflops = done * FLOP_PER_EVAL / (score_ms * 1e-3) / 1e12
    use_mf = bool(_lib.tune_get("score_mf")) and 2.0 ** -15 <= args.threshold < 1.0
    h, w = fhw
    s = 4 if cost_dtype == torch.float32 else 2
    if args.overlap_ref != "0":
        # the sweep kernel writes the warped half (and reads tgt); the reference
        # half (writes + its padded ref reads) is k_ref_planes' on the side stream
        sweep_bytes = B * (C * args.nlabel * h * w * s + C * h * w * 4)
        ref_bytes = B * (C * args.nlabel * h * w * s + C * h * w * 4)
    else:
        sweep_bytes = B * (2 * C * args.nlabel * h * w * s + 2 * C * h * w * 4)
    sweep_gbs = sweep_bytes / (kt["plane_sweep"] * 1e-3) / 1e9
    hyps = B * 512 * args.iters

    traffic, traffic_src = pmc_traffic(args)
    if rank == 0:
        pairs = world * B * args.steps
        corr = (f"{args.keypoints} SIFT-like keypoints" if args.keypoints
                else f"dense flow (N={hp.n}{', read by the RANSAC kernels' if hp.fused else ''})")
        out = {
            "metric": metric_name(args.nlabel, hwtxt),
            "value": round(pairs / elapsed, 3),
            "unit": "pairs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            **({"rehearsal": f"{world} ranks share one GPU over gloo (SFM_BENCH_SHARED_GPU): not a "
                              f"multi-GPU measurement"} if _shared_gpu() else {}),
            "src_hash": src_hash(),
            "dtype": "f64+" + ("f32" if s == 4 else "bf16"),
            "data": (f"synthetic (seeded {hwtxt.split()[0]}-shaped rigid scene, 0.5 px noise, 15% outlier flow, "
                     f"{corr}; N(0,1) features)"),
            "config": {"name": args.config,
                       "workload": (f"{hwtxt} {corr}, H={512 * args.iters} hypotheses (ransac_iter={args.iters}), "
                                    f"nlabel={args.nlabel}, C=32 at {h}x{w}, {args.cost_dtype} cost volume"),
                       "pairs_per_gpu": B, "global_batch": world * B, "parallelism": f"dp{world}",
                       "streams": "sweep on a side stream (overlaps the next step's solve)" if args.pipeline
                       else (f"reference half on a side stream ({args.overlap_ref})" if args.overlap_ref != "0"
                             else "one stream"),
                       **({"tune": args.tune} if args.tune else {})},
            "dist": {"world_size": torch.distributed.get_world_size() if torch.distributed.is_initialized() else 1,
                     "backend": torch.distributed.get_backend() if torch.distributed.is_initialized() else None,
                     "devices": names},
            "roofline": score_roofline(use_mf, score_tflops, done, evals, skipped, sum(cands), hp.n, score_ms,
                                       traffic.get("ransac_score"), traffic_src,
                                       rocprof_kernel_ms(args, ("k_mf_cands", "k_score_mf2"),
                                                         optional=("k_mf2_split", "k_mf2_lead", "k_mf2_keep",
                                                                   "k_mf2_keep_map", "k_mf2_zero_kept",
                                                                   "k_mf2_exact")),
                                       _lib.last_scorer(), upper_work),
            "roofline_sweep": {"kernel": "plane_sweep", "bound": "hbm", "achieved": round(sweep_gbs, 1),
                               "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": round(sweep_gbs / PEAK_HBM_GBS, 4),
                               "traffic": traffic.get("plane_sweep"), "traffic_source": traffic_src,
                               "avg_launch_ms": round(kt["plane_sweep"], 4),
                               "bytes_per_launch": sweep_bytes},
            "roofline_ref_planes": ({"kernel": "ref_planes (k_ref_pad + k_ref_planes, side stream beside the scorer)",
                                     "bound": "hbm", "avg_launch_ms": round(kt["ref_planes"], 4),
                                     "bytes_per_launch": ref_bytes,
                                     "achieved": round(ref_bytes / (kt["ref_planes"] * 1e-3) / 1e9, 1),
                                     "peak": PEAK_HBM_GBS, "unit": "GB/s",
                                     "note": "runs concurrently with k_score_mf2: its duration includes sharing "
                                             "the CUs with the scorer; not on the step's critical path"}
                                    if args.overlap_ref != "0" and "ref_planes" in kt else None),
            "solve": {"hypotheses_per_launch": hyps, "ms": round(kt_all["ransac_solve"], 4),
                      "hypotheses_per_s": round(hyps / (kt_all["ransac_solve"] * 1e-3), 1)},
            "kernel_ms": {k: round(v, 4) for k, v in {**kt_all, **kt}.items()},
            "kernel_ms_source": (f"{', '.join(ROOFLINE_REGIONS)}: HIP events in the timed region; the other stages: "
                                 f"HIP events around every stage in a separate pass of {min(args.steps, 5)} steps "
                                 f"after it (fully evented steps run the scorer slower, "
                                 f"{kt_all.get('ransac_score', 0.0):.3f} ms there)"),
            "inliers": [int(v) for v in gathered[:, 21].tolist()],
            "gathered": {"pairs": int(gathered.shape[0]), "per_rank": [len(dist.shard(world * B, r, world))
                                                                       for r in range(world)],
                         "via": "dist.gather_rows (all_gather of E[9], P[12], inliers per pair)"},
        }
        if world == 1 and not args.no_regularize and hp.cost.dtype in (torch.float32, torch.bfloat16):
            for prec, key in (("bf16", "roofline_regularize"), ("fp16", "roofline_regularize_fp16"),
                              ("fp32", "roofline_regularize_fp32"), ("fp32x3", "roofline_regularize_fp32x3")):
                try:
                    out[key] = regularize_roofline(hp.cost, steps=2 if prec == "fp32" else 3, precision=prec)
                except Exception as e:   # extra information, never the metric
                    out[key] = {"error": repr(e)}
        if world == 1 and not args.no_cpu_baseline:   # rank 0 at N=1 only
            try:
                out["cpu_baseline"] = cpu_baseline(flow, K, ref_fea, tgt_fea, P.float(), args,
                                                   n_pts=args.keypoints or None, keypoints=kp)
            except Exception as e:   # the baseline is reported, never the target
                out["cpu_baseline"] = {"value": None, "error": repr(e)}
        print(json.dumps(out), flush=True)
    if torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
