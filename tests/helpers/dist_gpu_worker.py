"""One rank of the two-rank GPU data-parallel check (tests/test_gpu_dist.py).

Started by tests/conftest.py as a fresh child process BEFORE the pytest
process touches the GPU (never an exec of a GPU-initialised process).  Every
rank builds the same seeded batch, runs TwoViewHotPath (HIP RANSAC + plane
sweep through libsfm_hip.so on cuda:0) on its own shard of the pairs
(sfm_amd.dist.shard), and the per-pair outputs (E, P, inliers and the whole
cost volume) are all-gathered with sfm_amd.dist.gather_rows (gloo); rank 0
writes them to $SFM_DIST_OUT/gathered.npy.  SURVEY.md §8(e)."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "deep-sfm-revisited_amd"))

# shared with the test's single-process run
PAIRS, HW, NLABEL, ITERS, THR, SEED = 5, (96, 160), 16, 2, 1e-3, 77


def make_inputs(device):
    from sfm_amd import synth
    flow, K, _, _ = synth.kitti_pair_batch(PAIRS, seed=SEED, hw=HW)
    fh, fw = synth.feature_hw(HW)
    r, t = synth.features(PAIRS, 32, fh, fw, seed=SEED)
    return [x.to(device) for x in (flow, K, r, t)]


def run(pair_ids, device):
    """Outputs of TwoViewHotPath for the given pairs: [n, 9 + 12 + 1 + cost] float64."""
    import torch
    from sfm_amd import synth
    from sfm_amd.pipeline import TwoViewHotPath
    flow, K, r, t = make_inputs(device)
    idx = torch.tensor(list(pair_ids), dtype=torch.long, device=device)
    n = len(pair_ids)
    hp = TwoViewHotPath(n, HW, synth.feature_hw(HW), 32, NLABEL, ITERS, THR, 1.0, rescale_depth=True,
                        device=device)
    E, P, inl, cost = hp.step(flow[idx], K[idx], r[idx], t[idx])
    torch.cuda.synchronize(device)
    return torch.cat([E.reshape(n, 9), P.reshape(n, 12), inl.reshape(n, 1).double(),
                      cost.reshape(n, -1).double()], 1).cpu()


def main():
    import numpy as np
    import torch
    from sfm_amd import dist
    rank, world, _ = dist.init(backend="gloo")
    dev = torch.device("cuda", 0)       # both ranks share the one GPU of the box
    torch.cuda.set_device(dev)
    mine = list(dist.shard(PAIRS, rank, world))
    rows = run(mine, dev)
    ids = torch.tensor(mine, dtype=torch.float64).reshape(-1, 1)
    allrows = dist.gather_rows(torch.cat([ids, rows], 1), world)
    if rank == 0:
        np.save(os.path.join(os.environ["SFM_DIST_OUT"], "gathered.npy"), allrows.numpy())
    torch.distributed.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
