"""World-size-2 coverage of the multi-GPU path on CPU (gloo): pairs shard
across ranks with no data-path collective, per-pair outputs are gathered to
every rank, timings reduce with max (sfm_amd/dist.py).

Each rank runs the oracle RANSAC on its shard of a small batch; the gathered
result must equal the single-process result, pair for pair."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _scene(seed, n=600):
    rng = np.random.default_rng(seed)
    X = np.c_[rng.uniform(-4, 4, n), rng.uniform(-2, 2, n), rng.uniform(6, 30, n)]
    a = rng.uniform(-0.03, 0.03, 3)
    Rx = np.array([[1, 0, 0], [0, np.cos(a[0]), -np.sin(a[0])], [0, np.sin(a[0]), np.cos(a[0])]])
    Ry = np.array([[np.cos(a[1]), 0, np.sin(a[1])], [0, 1, 0], [-np.sin(a[1]), 0, np.cos(a[1])]])
    R = Rx @ Ry
    t = np.array([0.1, 0.02, 1.0])
    Xp = X @ R.T + t
    q = X[:, :2] / X[:, 2:]
    qp = Xp[:, :2] / Xp[:, 2:]
    qp = qp + rng.normal(0, 2e-4, qp.shape)
    out = rng.random(n) < 0.2
    qp[out] = rng.uniform(-0.5, 0.5, (int(out.sum()), 2))
    return np.ascontiguousarray(q), np.ascontiguousarray(qp)


def _solve_pair(i):
    from oracle import ransac5 as ORR
    q, qp = _scene(100 + i)
    r = ORR.ransac5(q, qp, iters=2, thr=1e-3, nchains=64, nthreads=1)
    return np.r_[r["E"].ravel(), r["P"].ravel(), [r["inliers"], r["winner"]]]


def _worker(rank, world, port, num_pairs, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "deep-sfm-revisited_amd"))
    from sfm_amd import dist
    r, w, _ = dist.init(backend="gloo")
    assert (r, w) == (rank, world)
    mine = list(dist.shard(num_pairs, r, w))
    rows = torch.tensor(np.stack([_solve_pair(i) for i in mine]) if mine else np.zeros((0, 23)))
    ids = torch.tensor(mine, dtype=torch.float64).reshape(-1, 1)
    allrows = dist.gather_rows(torch.cat([ids, rows], 1), w)
    t = dist.reduce_max(float(rank + 1))
    dist.barrier()
    if rank == 0:
        np.save(out_path, np.c_[allrows.numpy(), np.full(allrows.shape[0], t)])
    torch.distributed.destroy_process_group()


def test_shard_covers_pairs_once():
    sys.path.insert(0, os.path.join(ROOT, "deep-sfm-revisited_amd"))
    from sfm_amd import dist
    for n in (0, 1, 5, 8, 33):
        for w in (1, 2, 3, 8):
            got = [i for r in range(w) for i in dist.shard(n, r, w)]
            assert got == list(range(n))
            sizes = [len(dist.shard(n, r, w)) for r in range(w)]
            assert max(sizes) - min(sizes) <= 1


@pytest.mark.parametrize("num_pairs", [5])
def test_two_rank_gloo_matches_single_process(tmp_path, num_pairs):
    out = str(tmp_path / "gathered.npy")
    mp.start_processes(_worker, args=(2, _free_port(), num_pairs, out), nprocs=2, join=True, start_method="spawn")
    got = np.load(out)
    assert got.shape[0] == num_pairs
    assert np.array_equal(got[:, 0], np.arange(num_pairs))          # rank order == pair order
    assert np.all(got[:, -1] == 2.0)                                 # max over ranks
    want = np.stack([_solve_pair(i) for i in range(num_pairs)])
    assert np.array_equal(got[:, 1:-1], want)                        # bit-identical per pair


def test_torchrun_world_of_one_gets_a_process_group():
    """Under torchrun (WORLD_SIZE and MASTER_PORT set) a world of 1 initialises
    the process group, so a one-GPU box runs the RCCL barrier / max-reduce
    path; a plain process (no torchrun variables) stays without one."""
    import subprocess
    code = ("import sys; sys.path.insert(0, {pkg!r}); import torch.distributed as d; "
            "from sfm_amd import dist; r = dist.init('gloo'); "
            "print(d.is_initialized(), r, dist.reduce_max(2.5))").format(
                pkg=os.path.join(ROOT, "deep-sfm-revisited_amd"))
    base = {k: v for k, v in os.environ.items()
            if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    launched = dict(base, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                    MASTER_PORT=str(_free_port()))
    out = subprocess.run([sys.executable, "-c", code], env=launched, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    last = out.stdout.strip().splitlines()[-1]          # gloo may log a line first
    assert last.split()[0] == "True" and last.endswith("2.5")
    out = subprocess.run([sys.executable, "-c", code], env=base, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert out.stdout.strip().splitlines()[-1].split()[0] == "False"
