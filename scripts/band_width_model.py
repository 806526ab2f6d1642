"""Experiment (CPU): how the width of k_score_mf2's decision band sets its
undecided rate.  The band's relative half-width is dominated by the AM-GM
slack delta of the certain-inlier / certain-outlier tests in score_mf.h
((|a| + alpha)^2 <= (1 + delta) a^2 + (1 + 1/delta) alpha^2), delta = 2^-6 in
round 2.  This replays k_mf_cands / mf_stage_point in numpy for candidate E's
of random 5-point samples on the bench's synthetic KITTI pair and counts the
evaluations with Ylo <= a'^2 <= Yhi for several delta.  a' and the D forms are
evaluated in float64 from the f16-rounded operands (the MFMA accumulation
error is inside eta), so the rates are a model of the kernel's, not a count
of it (the kernel's own count: SFM_MF_STATS builds)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "deep-sfm-revisited_amd"))
import torch  # noqa: E402
from oracle import ransac5 as ORR  # noqa: E402
from sfm_amd import synth  # noqa: E402

f16 = lambda v: np.asarray(v, np.float64).astype(np.float32).astype(np.float16).astype(np.float64)


def f16_up(v):
    return f16(np.asarray(v) * (1.0 + 2.0 ** -10) + 2.0 ** -24)


def points(seed, n_keep):
    flow, K, pose, _ = synth.kitti_pair_batch(1, seed=seed)
    Kinv = torch.inverse(K)[0].numpy()
    f = flow[0].numpy()                                   # [2, H, W]
    H, W = f.shape[1:]
    ys, xs = np.mgrid[0:H, 0:W]
    m = 10
    sel = (slice(m, H - m), slice(m, W - m))
    x0 = np.stack([xs[sel].ravel(), ys[sel].ravel(), np.ones(xs[sel].size)])
    x1 = np.stack([(xs + f[0])[sel].ravel(), (ys + f[1])[sel].ravel(), np.ones(xs[sel].size)])
    q = (Kinv @ x0)[:2].T
    qp = (Kinv @ x1)[:2].T
    rng = np.random.default_rng(seed)
    idx = rng.choice(q.shape[0], n_keep, replace=False)
    return q[idx], qp[idx]


def candidates(q, qp, n_samples, seed):
    rng = np.random.default_rng(seed + 7)
    out = []
    for _ in range(n_samples):
        i = rng.choice(q.shape[0], 5, replace=False)
        r = ORR.solve5(q[i], qp[i])
        out.extend(r["E"][:r["nP"]])
    return np.array(out)


def model(E, q, qp, thr, log2_inv_delta, acc_u=36):
    d = 2.0 ** -log2_inv_delta
    k = 0
    while k < 15 and np.ldexp(thr, k + 1) <= 1.0:
        k += 1
    t = np.ldexp(thr * thr, 2 * k)
    t_lo = t * (1 - 2.0 ** -40) * (1 - 2.0 ** -22) * (1 - 2.0 ** -18) / (1 + d)
    t_hi = t * (1 + 2.0 ** -40) * (1 + 2.0 ** -22) * (1 + 2.0 ** -18) / (1 - d)
    x, y, xp, yp = q[:, 0], q[:, 1], qp[:, 0], qp[:, 1]
    M = np.maximum(np.maximum(np.abs(x), np.abs(y)), np.maximum(np.abs(xp), np.abs(yp)))
    M = np.maximum(M, 1.0)
    ma = np.stack([xp * x, xp * y, xp, yp * x, yp * y, yp, x, y, np.ones_like(x)])
    md = np.stack([x * x, y * y, np.ones_like(x), x * y, x, y, xp * xp, yp * yp, xp * yp, xp, yp])
    s1 = ((np.abs(ma[0]) + np.abs(ma[1])) + (np.abs(ma[3]) + np.abs(ma[4]))) * 0.25
    s2 = ((np.abs(xp) + np.abs(yp)) + (np.abs(x) + np.abs(y))) * 0.25
    mon = np.concatenate([f16(md), f16_up(M * M)[None], f16_up(s1 * s1)[None], f16_up(s2 * s2)[None]])
    und = 0
    n_eval = 0
    for Ec in E:
        En = np.ldexp(Ec, -int(np.frexp(np.abs(Ec).max())[1]))
        cc = np.ldexp(En, k)
        a = cc @ ma
        e00, e01, e02, e10, e11, e12, e20, e21 = En[:8]
        g = np.array([e00 * e00 + e10 * e10, e01 * e01 + e11 * e11,
                      (e02 * e02 + e12 * e12) + (e20 * e20 + e21 * e21), 2 * (e00 * e01 + e10 * e11),
                      2 * (e00 * e02 + e10 * e12), 2 * (e01 * e02 + e11 * e12), e00 * e00 + e01 * e01,
                      e10 * e10 + e11 * e11, 2 * (e00 * e10 + e01 * e11), 2 * (e00 * e20 + e01 * e21),
                      2 * (e10 * e20 + e11 * e21)])
        kacc = acc_u * 2.0 ** -24
        aS = kacc * (1 + 2.0 ** -9) + 3.75 * 2.0 ** -22 + kacc * 2.0 ** -8 + 2.0 ** -46
        C1 = max(abs(cc[0]), abs(cc[1]), abs(cc[3]), abs(cc[4]))
        C2 = max(abs(cc[2]), abs(cc[5]), abs(cc[6]), abs(cc[7]))
        K1 = aS * C1 + 2.0 ** -24
        K2 = aS * C2 + 2.0 ** -24
        K3 = aS * abs(cc[8]) + 2.0 ** -24 + 9 * 2.0 ** -24 * np.abs(cc).max()
        infl = 3 * (1 + 2.0 ** -9)
        p_in, p_out = 1 + 1 / d, 1 / d
        e1 = np.array([16 * infl * p_in * K1 * K1, 16 * infl * p_in * K2 * K2, infl * p_in * K3 * K3]) / (1 + d)
        e2 = np.array([16 * infl * p_out * K1 * K1, 16 * infl * p_out * K2 * K2, infl * p_out * K3 * K3]) / (1 - d)
        gl = f16(t_lo * g)
        gh = f16(t_hi * g)
        gl[2] = f16(t_lo * g[2] - e1[2])
        gh[2] = f16(t_hi * g[2] + e2[2])
        eta_lo = (1.048e-3 * np.abs(gl).sum() + 11 * 2.0 ** -25 * (np.abs(gl).max() + 1)) * (1 + 2.0 ** -9)
        eta_hi = (1.048e-3 * np.abs(gh).sum() + 11 * 2.0 ** -25 * (np.abs(gh).max() + 1)) * (1 + 2.0 ** -9)
        rl = np.concatenate([gl, [-f16_up(eta_lo), -f16_up(e1[0]), -f16_up(e1[1])]])
        rh = np.concatenate([gh, [f16_up(eta_hi), f16_up(e2[0]), f16_up(e2[1])]])
        Ylo = rl @ mon
        Yhi = rh @ mon
        aa = a * a
        und += int(np.count_nonzero((aa >= Ylo) & (aa <= Yhi)))
        n_eval += a.size
    return und / n_eval


if __name__ == "__main__":
    q, qp = points(1000, 20000)
    E = candidates(q, qp, 150, 1000)
    print("%d candidates x %d points" % (len(E), q.shape[0]))
    for thr in (1e-4, 1e-3):
        for l in (6, 7, 8, 9, 10):
            print("thr %g  delta 2^-%d  undecided %.4f %%" % (thr, l, 100 * model(E, q, qp, thr, l)))
