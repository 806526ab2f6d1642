"""Experiment (CPU): undecided rate of a single-band scorer (DESIGN.md §7,
the round-5 candidate) against today's two-sided band, in float64 on a
synthetic KITTI-like pair (oracle/gen_golden.geometric_scene) with the
candidates of random 5-point samples (oracle solve5).

Today (k_score_mf2): undecided iff |a^2 - Y| < delta * Y (+ the split-f16 /
accumulation error terms, ignored here), a = q'^T E q, Y = thr^2 D, D =
(Eq)_0^2 + (Eq)_1^2 + (E^T q')_0^2 + (E^T q')_1^2, delta = 2^-5.

Single band: one output u = (a^2 - Y) / S with S = f(c) g(p) separable and
f g >= delta * Y for every (c, p); undecided iff |a^2 - Y| < 2 S (the
|u| >= 2 exponent bit).  Two separable bounds:
  * Cauchy-Schwarz: D <= max(|E_0|^2 + |E_1|^2, |E^0|^2 + |E^1|^2) (|q|^2 + |q'|^2)
    (row / column norms of E), f = delta thr^2 max(...), g = |q|^2 + |q'|^2;
  * per-candidate exact max over the point set ("oracle" in g = 1): f(c) =
    delta thr^2 max_p D(c, p) -- a per-candidate uniform band.
usage: python scripts/single_band_model.py [thr] [n_points] [n_samples]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import ransac5 as R  # noqa: E402
from oracle.gen_golden import geometric_scene  # noqa: E402

thr = float(sys.argv[1]) if len(sys.argv) > 1 else 1e-4
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
ns = int(sys.argv[3]) if len(sys.argv) > 3 else 200
delta = 2.0 ** -5
rng = np.random.default_rng(7)
q, qp = geometric_scene(rng, n, out_frac=0.15, noise=0.001)
Es = []
for _ in range(ns):
    idx = rng.choice(n, 5, replace=False)
    r = R.solve5(q[idx], qp[idx], cheir=True)
    Es += [r["E"][j].reshape(3, 3) for j in range(int(r["nP"]))]
Es = np.array(Es)
Q = np.concatenate([q, np.ones((n, 1))], 1)
QP = np.concatenate([qp, np.ones((n, 1))], 1)
tot = {"today": 0, "cs": 0, "uniform": 0}
inl = 0
for E in Es:
    Eq = Q @ E.T                      # rows: E q
    EtQ = QP @ E                      # rows: E^T q'
    a = np.einsum("ij,ij->i", QP, Eq)
    D = Eq[:, 0] ** 2 + Eq[:, 1] ** 2 + EtQ[:, 0] ** 2 + EtQ[:, 1] ** 2
    Y = thr * thr * D
    gap = np.abs(a * a - Y)
    inl += int((a * a <= Y).sum())
    tot["today"] += int((gap < delta * Y).sum())
    fc = max((E[0] ** 2).sum() + (E[1] ** 2).sum(), (E[:, 0] ** 2).sum() + (E[:, 1] ** 2).sum())
    gp = (Q ** 2).sum(1) + (QP ** 2).sum(1)
    tot["cs"] += int((gap < 2 * delta * thr * thr * fc * gp).sum())
    tot["uniform"] += int((gap < 2 * delta * Y.max()).sum())
ev = len(Es) * n
print(f"thr {thr:g}: {len(Es)} candidates x {n} points, inlier rate {inl / ev:.4f}")
for k, v in tot.items():
    print(f"  {k:8s} undecided {100.0 * v / ev:.3f} %")
