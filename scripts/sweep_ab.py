"""Same-process A/B of sweep tuning keys on the bench volume (KITTI B pairs,
L=128, 94x311, C=32): per-launch plane_sweep time from the library's HIP-event
profiler, 10 launches per variant and round, three interleaved rounds; every
variant's volume must equal the first variant's bit for bit.  AB_ROUNDS
rounds (default 3), odd rounds in reverse variant order.
Usage: sweep_ab.py [dtype=bf16] [B=4] "k=v,k=v" "k=v" ..."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deep-sfm-revisited_amd"))
import torch
from sfm_amd import _lib, synth
from sfm_amd import sweep as SW

dtype, B, names = torch.float32, 8, []
ROUNDS = int(os.environ.get("AB_ROUNDS", "3"))
for a in sys.argv[1:]:
    if a.startswith("dtype="):
        dtype = torch.bfloat16 if a.split("=")[1] == "bf16" else torch.float32
    elif a.startswith("B="):
        B = int(a.split("=")[1])
    else:
        names.append(a)
names = names or [""]
variants = [dict(kv.split("=") for kv in v.split(",") if kv) for v in names]
dev = torch.device("cuda", 0)
C, L, h, w = 32, 128, 94, 311
_, K, pose, _ = synth.kitti_pair_batch(B, seed=1000, device=dev)
ref, tgt = synth.features(B, C, h, w, device=dev)
K4, Ki4 = SW.quarter_intrinsics(K, torch.inverse(K))
P = pose[:, :3, :4].float().contiguous().to(dev)
out = torch.empty(B, 2 * C, L, h, w, device=dev, dtype=dtype)
ws = SW.workspace_for(B, C, h, w, dev)
nbytes = out.numel() * out.element_size() + ref.numel() * 4 + tgt.numel() * 4
res = {i: [] for i in range(len(variants))}
base = None
for rnd in range(ROUNDS):
    order = list(enumerate(variants))
    for i, v in (order if rnd % 2 == 0 else order[::-1]):
        for k, x in v.items():
            _lib.tune(k, int(x))
        out.fill_(float("nan"))
        SW.plane_sweep_cost(ref, tgt, P, K4, Ki4, L, 1.0, dtype=dtype, out=out, workspace=ws)
        torch.cuda.synchronize()
        if base is None:
            base = out.clone()
        assert torch.equal(base.view(torch.int16 if dtype == torch.bfloat16 else torch.int32),
                           out.view(torch.int16 if dtype == torch.bfloat16 else torch.int32)), \
            f"variant {names[i]} changed the volume"
        _lib.profile_reset(); _lib.profile_enable(True)
        for _ in range(10):
            SW.plane_sweep_cost(ref, tgt, P, K4, Ki4, L, 1.0, dtype=dtype, out=out, workspace=ws)
        torch.cuda.synchronize(); _lib.profile_enable(False)
        ms, n = _lib.profile_read("plane_sweep")
        res[i].append(ms / max(n, 1))
for i in range(len(variants)):
    r = sorted(res[i])
    med = r[len(r) // 2]
    print(f"{str(dtype)[6:]:9s} B={B} {names[i] or 'default':28s} sweep median {med:.4f} ms "
          f"({nbytes / (med * 1e-3) / 1e9:.0f} GB/s)  all {[round(x, 4) for x in res[i]]}", flush=True)
