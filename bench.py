#!/usr/bin/env python3
"""Benchmark: image-pairs/sec of the two-view SfM hot path on MI355X.

One step = one batch of `--batch` KITTI-shaped pairs (376x1242 dense flow,
N = 435,032 correspondences) per GPU through
    flow -> correspondences -> RANSAC five-point (H = 512 x iters = 4096)
    -> pose (RESCALE_DEPTH, NORM_TARGET 0.6) -> plane-sweep cost volume
       [B, 64, 128, 94, 311] fp32
with every input already resident in HBM (BASELINE.json configs[1]).
Multi-GPU: one process per GPU (torchrun), pairs shard across ranks with no
data-path collective ("scaling": "weak"); RCCL only for the barrier and the
max-over-ranks timing reduction.

Rank 0 prints ONE JSON line.  `roofline` is the dominant kernel (RANSAC
scoring, fp64 VALU); `roofline_sweep` the HBM-bound cost-volume kernel; both
average launch durations come from HIP events recorded by libsfm_hip around
every launch on the launching stream during the timed region; `traffic` is
the PMC-measured HBM bytes per launch (FETCH_SIZE x2 + WRITE_SIZE, gfx950
correction) from the committed profiles/rNN_pmc.json of the same workload.  The
`cpu_baseline` is the oracle (CPU restatement) on a bounded sample, rank 0 at N=1 only.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "deep-sfm-revisited_amd"))

import torch  # noqa: E402

from sfm_amd import _lib, dist, ransac, synth  # noqa: E402
from sfm_amd.pipeline import TwoViewHotPath  # noqa: E402

PEAK_HBM_GBS = 8000.0        # MI355X HBM3E spec (MI355X_MICROARCH.md)
PEAK_FP64_TFLOPS = 78.6      # MI355X fp64 vector spec
PEAK_FP32_TFLOPS = 157.3     # MI355X fp32 vector spec (MI355X_MICROARCH.md)
PEAK_BF16_TFLOPS = 2500.0    # MI355X dense bf16 MFMA (MI355X_MICROARCH.md; no sparsity)
FLOP_PER_EVAL = 50           # Ex, xE, x'Ex, sqrt, div, |.|


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=8, help="pairs per GPU per step")
    ap.add_argument("--nlabel", type=int, default=128)
    ap.add_argument("--iters", type=int, default=8, help="ransac_iter (H = 512 x iters)")
    ap.add_argument("--threshold", type=float, default=1e-4)
    ap.add_argument("--cost-dtype", choices=["fp32", "bf16"], default="fp32")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-regularize", action="store_true",
                    help="skip the (unscored) PSNet 3-D regularisation roofline line after the timed region")
    ap.add_argument("--fused", action="store_true",
                    help="RANSAC reads the flow directly (sfm_ransac5_flow) instead of materialised correspondences")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--pipeline", action="store_true",
                    help="sweep on a side stream, overlapping the next step's solve (measured slower: 460 vs 466 pairs/s)")
    return ap.parse_args()


def pmc_traffic(args):
    """HBM bytes per launch of the path's kernels from the newest committed PMC
    summary (profiles/rNN_pmc.json, scripts/gpu_pmc.sh + scripts/pmc_summary.py;
    counters need their own profiler pass, so they cannot be read live here).
    Only reported for the default workload the summary was collected on."""
    import glob
    if (args.batch, args.nlabel, args.iters, args.cost_dtype) != (8, 128, 8, "fp32"):
        return {}, None
    fs = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc*.json")))
    if not fs:
        return {}, None
    k = json.load(open(fs[-1]))["kernels"]
    return {n: v.get("hbm_bytes") for n, v in k.items()}, os.path.relpath(fs[-1], ROOT)


def cpu_baseline(flow, K, ref_fea, tgt_fea, pose, args):
    """Oracle (CPU restatement) on a bounded sample of the same workload:
    one pair, RANSAC with 64 chains x `iters` (of 512) hypotheses on all
    435,032 correspondences, and the sweep on 16 of 128 planes; both scaled to
    one full pair."""
    import numpy as np
    sys.path.insert(0, ROOT)
    from oracle import ransac5 as ORR
    from oracle import sweep as OSW
    threads = max(1, min(args.cpu_threads, len(os.sched_getaffinity(0))))
    torch.set_num_threads(threads)
    Kinv = torch.inverse(K[:1].cpu())
    pts = ransac.flow_to_points(flow[:1], Kinv.to(flow.device)).cpu().numpy()[0]
    q, qp = np.ascontiguousarray(pts[:, :2]), np.ascontiguousarray(pts[:, 2:])
    chains = 64
    ORR.ransac5(q[:2000], qp[:2000], iters=1, thr=args.threshold, nchains=8, nthreads=threads)   # warm-up
    t0 = time.perf_counter()
    ORR.ransac5(q, qp, iters=args.iters, thr=args.threshold, nchains=chains, nthreads=threads)
    t_ransac = (time.perf_counter() - t0) * (512 / chains)
    planes = list(range(0, args.nlabel, max(1, args.nlabel // 16)))
    r = ref_fea[:1].cpu(); t = tgt_fea[:1].cpu(); P = pose[:1].cpu(); Kc = K[:1].cpu()
    OSW.plane_sweep_cost(r, t, P, Kc, torch.inverse(Kc), args.nlabel, 1.0, rescale=0.6, planes=planes[:2])
    t0 = time.perf_counter()
    OSW.plane_sweep_cost(r, t, P, Kc, torch.inverse(Kc), args.nlabel, 1.0, rescale=0.6, planes=planes)
    t_sweep = (time.perf_counter() - t0) * (args.nlabel / len(planes))
    per_pair = t_ransac + t_sweep
    return {"value": round(1.0 / per_pair, 4), "unit": "pairs/s", "cores": threads, "kind": "port",
            "sample": (f"1 KITTI pair: RANSAC {chains}/512 chains x {args.iters} iters on N=435032 "
                       f"({t_ransac:.2f} s/pair scaled), sweep {len(planes)}/{args.nlabel} planes "
                       f"({t_sweep:.3f} s/pair scaled), oracle C++ (OpenMP) + torch-CPU fp32")}


def regularize_roofline(cost, steps=3):
    """PSNet's 12-layer 3-D cost regularisation (sfm_conv3_bf16) on the first
    pair of the last step's cost volume, after the timed region.  Not part of
    ``value`` (the metric's path ends at the cost volume); reported so the
    MFMA kernel's roofline is measured live beside the path's."""
    from sfm_amd.regularize import CostRegularization
    torch.manual_seed(0)
    reg = CostRegularization(cost.shape[1]).to(cost.device).eval()
    one = cost[:1]
    reg(one)
    torch.cuda.synchronize(cost.device)
    _lib.profile_reset()
    _lib.profile_enable(True)
    for _ in range(steps):
        reg(one)
    torch.cuda.synchronize(cost.device)
    _lib.profile_enable(False)
    ms, n = _lib.profile_read("conv3")
    _, L, h, w = one.shape[1:]
    vox = L * h * w
    flop = 2 * vox * 27 * (one.shape[1] * 32 + 10 * 32 * 32 + 32)
    per_stack = ms / steps
    tf = flop / (per_stack * 1e-3) / 1e12
    return {"kernel": "conv3 x12 (PSNet dres0..classify, bf16 MFMA)", "bound": "mfma-bf16", "achieved": round(tf, 1),
            "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s", "frac": round(tf / PEAK_BF16_TFLOPS, 4),
            "avg_launch_ms": round(ms / max(n, 1), 4), "ms_per_stack": round(per_stack, 4),
            "work": f"{flop} FLOP per stack (1 pair, L={L}, {h}x{w}; 2*27*Cin*Cout per voxel and layer)",
            "note": "not part of value: the CNN after the measured path, timed after it"}


def main():
    args = parse()
    rank, world, local = dist.init()
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    B = args.batch
    hw = synth.KITTI_HW
    fhw = synth.feature_hw(hw)
    C = 32
    cost_dtype = torch.float32 if args.cost_dtype == "fp32" else torch.bfloat16

    # synthetic inputs, distinct pairs per rank, resident in HBM before timing
    flow, K, pose_gt, _ = synth.kitti_pair_batch(B, seed=1000 + rank, hw=hw, device=dev)
    ref_fea, tgt_fea = synth.features(B, C, fhw[0], fhw[1], seed=rank, device=dev)
    hp = TwoViewHotPath(B, hw, fhw, C, args.nlabel, args.iters, args.threshold, 1.0, rescale_depth=True,
                        norm_target=0.6, cost_dtype=cost_dtype, device=dev, fused=args.fused)

    # --pipeline: step i's sweep (side stream) overlaps step i+1's five-point solve
    stepf = hp.step_pipelined if args.pipeline else hp.step
    for _ in range(args.warmup):
        stepf(flow, K, ref_fea, tgt_fea)
    torch.cuda.synchronize(dev)
    _lib.profile_reset()
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

    kt = {}
    for name in ("flow_to_points", "ransac_solve", "ransac_chain", "ransac_score", "ransac_select", "plane_sweep"):
        ms, n = _lib.profile_read(name)
        kt[name] = ms / max(n, 1)
    cands = ransac.candidate_counts(hp.ws, B, args.iters)
    if hp.fused:
        kt.pop("flow_to_points", None)
    evals = sum(cands) * hp.n                       # candidate E x correspondences per launch
    skipped = ransac.skipped_evaluations(hp.ws, B, args.iters)   # exact bound pruning (last launch)
    done = evals - skipped                          # evaluations the launch performed
    score_ms = kt["ransac_score"]
    score_tflops = done * FLOP_PER_EVAL / (score_ms * 1e-3) / 1e12
    h, w = fhw
    s = 4 if cost_dtype == torch.float32 else 2
    sweep_bytes = B * (2 * C * args.nlabel * h * w * s + 2 * C * h * w * 4)
    sweep_gbs = sweep_bytes / (kt["plane_sweep"] * 1e-3) / 1e9

    traffic, traffic_src = pmc_traffic(args)
    if rank == 0:
        pairs = world * B * args.steps
        out = {
            "metric": "image-pairs/sec (5-pt RANSAC + nlabel=128 plane-sweep), KITTI 376x1242",
            "value": round(pairs / elapsed, 3),
            "unit": "pairs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64+" + ("f32" if s == 4 else "bf16"),
            "data": "synthetic (seeded KITTI-shaped rigid scene, 0.5 px noise, 15% outlier flow; N(0,1) features)",
            "config": {"workload": (f"KITTI 376x1242 dense flow (N={hp.n}), H={512 * args.iters} hypotheses "
                                    f"(ransac_iter={args.iters}), nlabel={args.nlabel}, C=32 at 94x311, "
                                    f"{args.cost_dtype} cost volume"),
                       "pairs_per_gpu": B, "global_batch": world * B, "parallelism": f"dp{world}",
                       "streams": "sweep on a side stream (overlaps the next step's solve)" if args.pipeline
                       else "one stream"},
            # k_score32 decides ~99% of evaluations in float32 (the rest re-tested in
            # float64), so the binding peak is the float32 VALU one
            "roofline": {"kernel": "ransac_score", "bound": "valu-fp32", "achieved": round(score_tflops, 3),
                         "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s", "frac": round(score_tflops / PEAK_FP32_TFLOPS, 4),
                         "traffic": traffic.get("ransac_score"), "traffic_source": traffic_src,
                         "avg_launch_ms": round(score_ms, 4),
                         "work": (f"{done} evals x {FLOP_PER_EVAL} FLOP per launch: {sum(cands)} candidate E x "
                                  f"N={hp.n} = {evals}, minus {skipped} skipped by exact bound pruning "
                                  f"({100.0 * skipped / max(evals, 1):.1f}%)")},
            "roofline_sweep": {"kernel": "plane_sweep", "bound": "hbm", "achieved": round(sweep_gbs, 1),
                               "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": round(sweep_gbs / PEAK_HBM_GBS, 4),
                               "traffic": traffic.get("plane_sweep"), "traffic_source": traffic_src,
                               "avg_launch_ms": round(kt["plane_sweep"], 4),
                               "bytes_per_launch": sweep_bytes},
            "kernel_ms": {k: round(v, 4) for k, v in kt.items()},
            "inliers": [int(v) for v in inl.cpu()],
        }
        if world == 1 and not args.no_regularize and hp.cost.dtype in (torch.float32, torch.bfloat16):
            try:
                out["roofline_regularize"] = regularize_roofline(hp.cost)
            except Exception as e:   # extra information, never the metric
                out["roofline_regularize"] = {"error": repr(e)}
        if world == 1 and not args.no_cpu_baseline:   # rank 0 at N=1 only
            try:
                out["cpu_baseline"] = cpu_baseline(flow, K, ref_fea, tgt_fea, P.float(), args)
            except Exception as e:   # the baseline is reported, never the target
                out["cpu_baseline"] = {"value": None, "error": repr(e)}
        print(json.dumps(out), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
