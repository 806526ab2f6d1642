"""The product's multi-rank path on the GPU (main.py:219):
two fresh ranks (tests/helpers/dist_gpu_worker.py, gloo, both on cuda:0,
started by conftest.py before this process touched the GPU) each run the HIP
hot path (TwoViewHotPath: RANSAC five-point + plane sweep) on their shard of
5 pairs (3 + 2) and all-gather E, P, inliers and the cost volume.  The
gathered outputs must equal one single-process run over all 5 pairs, bit for
bit."""
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "helpers"))


@pytest.mark.gpu
def test_two_ranks_gather_equals_single_process(dist_gpu_ranks, cuda):
    import dist_gpu_worker as W
    procs, out_dir = dist_gpu_ranks
    for p in procs:
        try:
            rc = p.wait(timeout=90)
        except Exception:
            p.kill()
            raise
        assert rc == 0, f"rank exited with {rc}: " + open(os.path.join(out_dir, f"rank{procs.index(p)}.log")).read()[-3000:]
    got = np.load(os.path.join(out_dir, "gathered.npy"))
    assert got.shape[0] == W.PAIRS
    assert list(got[:, 0]) == list(range(W.PAIRS))          # rank order = pair order
    want = W.run(range(W.PAIRS), cuda).numpy()
    assert np.array_equal(got[:, 1:], want)
    assert (want[:, 21] > 0).all()                          # every pair found inliers
