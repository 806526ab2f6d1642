"""Probe (round 3): which float32 LU + triangular-solve operation order
(scripts/probe_kinv.hip, 64 variants) reproduces torch.linalg.inv_ex on this
ROCm build bit for bit, for intrinsic matrices (zero skew, K22 = 1) and for
general 3x3 matrices.  Prints, per variant, the matrices that differ."""
import ctypes, os, sys
import torch
HERE = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(HERE, "exp", "probe_kinv.so"))
dev = torch.device("cuda", 0)
g = torch.Generator().manual_seed(7)
n = 20000
fx = 100 + 1900 * torch.rand(n, generator=g)
fy = fx * (0.8 + 0.4 * torch.rand(n, generator=g))
cx = 2500 * torch.rand(n, generator=g)   # |cx| > fx in part: pivoting
cy = 1500 * torch.rand(n, generator=g)
K = torch.zeros(n, 3, 3)
K[:, 0, 0], K[:, 0, 2], K[:, 1, 1], K[:, 1, 2], K[:, 2, 2] = fx, cx, fy, cy, 1.0
G = torch.randn(n, 3, 3, generator=g) * torch.exp(torch.randn(n, 1, 1, generator=g))
for name, A in (("intrinsics", K), ("general", G)):
    A = A.float().contiguous().to(dev)
    want = torch.linalg.inv_ex(A)[0]
    nmode = 64
    out = torch.empty(nmode, n, 3, 3, dtype=torch.float32, device=dev)
    assert lib.probe_kinv(ctypes.c_void_p(A.data_ptr()), n, nmode, ctypes.c_void_p(out.data_ptr())) == 0
    wb = want.view(torch.int32)
    res = []
    for m in range(nmode):
        bad = (out[m].view(torch.int32) != wb).reshape(n, 9).any(1).sum().item()
        res.append((bad, m))
    res.sort()
    print(name, "best variants (mismatching matrices, mode):", res[:8], flush=True)
    for m in sorted(set([39] + [r[1] for r in res[:3]])):
        o = out[m]
        val = (o != want).reshape(n, 9).any(1).sum().item()                 # value mismatches (+0 == -0)
        bits = (o.view(torch.int32) != wb).reshape(n, 9)
        zs = (bits & (o == want).reshape(n, 9)).sum(0).tolist()                            # entries differing only in a zero's sign
        print("  mode %d: value mismatches %d, zero-sign-only differences per entry %s" % (m, val, zs), flush=True)
        if bits.any():
            k = int(bits.any(1).nonzero()[0])
            print("    e.g.", A[k].tolist(), "torch", want[k].tolist(), "mode", o[k].tolist(), flush=True)
