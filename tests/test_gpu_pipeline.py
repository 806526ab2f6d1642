"""bench.py --pipeline: TwoViewHotPath.step_pipelined runs each step's plane
sweep on a side stream, overlapping the next step's pose stage (and, with the
score gate, not its scorer).  Steps issued back to back (so the overlap
really happens) must give the same E, P, inlier counts and cost volume as
plain sequential steps; the reference-half overlap and the score fence are
tested below."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("gate", [True, False])
def test_pipelined_steps_equal_plain_steps(cuda, gate):
    from sfm_amd import synth
    from sfm_amd.pipeline import TwoViewHotPath
    B, C, L, fhw = 2, 32, 32, (94, 311)
    steps = []
    for s in (11, 12, 13):
        flow, K, _, _ = synth.kitti_pair_batch(B, seed=s, device=cuda)
        ref, tgt = synth.features(B, C, *fhw, seed=s, device=cuda)
        steps.append((flow, K, ref, tgt))
    mk = lambda: TwoViewHotPath(B, (376, 1242), fhw, C, L, 2, 1e-4, 1.0, True, 0.6, device=cuda, gate_scorer=gate)
    plain, piped = mk(), mk()
    outs = [piped.step_pipelined(*a) for a in steps]      # back to back: sweep i overlaps pose i+1
    torch.cuda.synchronize()
    for a, o in zip(steps, outs):
        E, P, inl, _ = plain.step(*a)
        assert torch.equal(E, o[0]) and torch.equal(P, o[1]) and torch.equal(inl, o[2])
    torch.cuda.synchronize()
    assert torch.equal(plain.cost, piped.cost)            # the last step's volume


@pytest.mark.parametrize("dtype,fhw,L,mode", [(torch.float32, (94, 311), 32, "score"),
                                               (torch.bfloat16, (94, 311), 16, "score"),
                                               (torch.float32, (94, 311), 16, "step"),
                                               (torch.float32, (20, 30), 8, "score"),
                                               (torch.float32, (12, 17), 5, "step")])
def test_overlapped_reference_half_equals_full_sweep(cuda, dtype, fhw, L, mode):
    """step_overlap: the reference half from sfm_plane_sweep_ref_planes on a
    side stream behind the score fence, the warped half from
    sfm_plane_sweep_psnet_warped_half.  Steps back to back; the volume must
    equal the one-launch sweep's bit for bit, at KITTI size (fast copy path)
    and at small / odd shapes (generic path: hw < the padding, L * hw % 64 != 0)."""
    from sfm_amd import synth
    from sfm_amd.pipeline import TwoViewHotPath
    B, C = 2, 32
    steps = []
    for s in (21, 22):
        flow, K, _, _ = synth.kitti_pair_batch(B, seed=s, device=cuda)
        ref, tgt = synth.features(B, C, *fhw, seed=s, device=cuda)
        steps.append((flow, K, ref, tgt))
    mk = lambda ov: TwoViewHotPath(B, (376, 1242), fhw, C, L, 2, 1e-4, 1.0, True, 0.6, cost_dtype=dtype,
                                   device=cuda, overlap_ref=ov)
    plain, over = mk(False), mk(mode)
    for a in steps:
        over.cost.fill_(float("nan"))                       # every element must be written this step
        E2, P2, i2, c2 = over.step(*a)
        E1, P1, i1, c1 = plain.step(*a)
        torch.cuda.synchronize()
        assert torch.equal(E1, E2) and torch.equal(P1, P2) and torch.equal(i1, i2)
        assert torch.equal(c1, c2)


def test_ref_planes_alone_write_only_the_reference_rows(cuda):
    from sfm_amd import sweep, synth
    B, C, L, h, w = 3, 32, 16, 94, 311
    ref, _ = synth.features(B, C, h, w, seed=5, device=cuda)
    out = torch.full((B, 2 * C, L, h, w), 7.0, device=cuda)
    sweep.plane_sweep_ref_half(ref, L, out)
    torch.cuda.synchronize()
    assert torch.equal(out[:, :C], ref.unsqueeze(2).expand(B, C, L, h, w))
    assert bool((out[:, C:] == 7.0).all())


def test_score_fence_per_device_and_released(cuda):
    """The score fence lives on the device of the stream it is recorded on and
    stays enabled while any overlap_ref hot path lives: a second hot path's
    release leaves the first one's steps working, and after the last one is
    gone waiting is refused (reference count back to zero)."""
    import gc
    from sfm_amd import _lib, synth
    from sfm_amd.pipeline import TwoViewHotPath
    B, C, L, fhw = 1, 32, 8, (20, 30)
    flow, K, _, _ = synth.kitti_pair_batch(B, seed=31, hw=(120, 200), device=cuda)
    ref, tgt = synth.features(B, C, *fhw, seed=31, device=cuda)
    mk = lambda ov: TwoViewHotPath(B, (120, 200), fhw, C, L, 2, 1e-3, 1.0, True, 0.6, device=cuda, overlap_ref=ov)
    gc.collect()
    before = _lib.load().sfm_score_fence_wait(_lib.stream_ptr(cuda))   # 1 unless an earlier hot path still lives
    a, b = mk("score"), mk("score")
    del b
    gc.collect()
    plain = mk(False)
    E2, P2, i2, c2 = a.step(flow, K, ref, tgt)
    E1, P1, i1, c1 = plain.step(flow, K, ref, tgt)
    torch.cuda.synchronize()
    assert torch.equal(c1, c2) and torch.equal(E1, E2)
    del a
    gc.collect()
    assert _lib.load().sfm_score_fence_wait(_lib.stream_ptr(cuda)) == before


@pytest.mark.skipif(not torch.cuda.is_available() or torch.cuda.device_count() < 2, reason="needs two GPUs")
def test_overlap_hot_path_on_non_current_device():
    """a hot path built for a device other than the current one
    records and waits on that device's own fence."""
    from sfm_amd import synth
    from sfm_amd.pipeline import TwoViewHotPath
    dev = torch.device("cuda", 1)
    torch.cuda.set_device(0)
    B, C, L, fhw = 1, 32, 8, (20, 30)
    flow, K, _, _ = synth.kitti_pair_batch(B, seed=32, hw=(120, 200), device=dev)
    ref, tgt = synth.features(B, C, *fhw, seed=32, device=dev)
    over = TwoViewHotPath(B, (120, 200), fhw, C, L, 2, 1e-3, 1.0, True, 0.6, device=dev, overlap_ref="score")
    plain = TwoViewHotPath(B, (120, 200), fhw, C, L, 2, 1e-3, 1.0, True, 0.6, device=dev)
    with torch.cuda.device(dev):
        c2 = over.step(flow, K, ref, tgt)[3]
        c1 = plain.step(flow, K, ref, tgt)[3]
        torch.cuda.synchronize(dev)
    assert torch.equal(c1, c2)


def test_score_gate_one_shot(cuda):
    """sfm_score_gate(stream, 1) records the library's gate event on a side
    stream and arms it: the next RANSAC call on the device holds its scoring
    phase until the side stream reaches that point, and disarms the gate; the
    call after it does not wait; arm = 0 disarms without waiting."""
    import ctypes
    from sfm_amd import _lib, synth
    lib = _lib.load()
    B = 2
    flow, K, _, _ = synth.kitti_pair_batch(B, seed=5, device=cuda)
    from sfm_amd.pipeline import TwoViewHotPath
    hp = TwoViewHotPath(B, (376, 1242), (94, 311), 32, 8, device=cuda)
    Kinv = hp.k_inverse(K)
    hp.pose(flow, K, Kinv)                                   # warm: kernels loaded, buffers touched
    torch.cuda.synchronize()
    side = torch.cuda.Stream(device=cuda)
    main = torch.cuda.current_stream(cuda)

    def timed_pose(sleep_cycles, arm):
        with torch.cuda.stream(side):
            torch.cuda._sleep(sleep_cycles)
        if arm is not None:
            assert lib.sfm_score_gate(ctypes.c_void_p(side.cuda_stream), ctypes.c_void_p(main.cuda_stream), arm) == 0
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record(main)
        hp.pose(flow, K, Kinv)
        t1.record(main)
        torch.cuda.synchronize()
        return t0.elapsed_time(t1)

    base = timed_pose(1000, None)                            # no gate: the pose stage alone
    sleep = 200_000_000                                      # ~0.1 s on the side stream
    gated = timed_pose(sleep, 1)
    assert gated > base + 20.0, (base, gated)                # held for the side stream
    free = timed_pose(sleep, None)                           # the gate was consumed
    assert free < base + 20.0, (base, free)
    disarmed = timed_pose(sleep, 0)                          # arm = 0: nothing to wait for
    assert disarmed < base + 20.0, (base, disarmed)


def test_score_gate_scoped_to_its_waiting_stream(cuda):
    """The gate is armed for one waiting stream: a RANSAC call on another
    stream of the same device (a second hot path, a plain computeP) neither
    waits for it nor consumes it; the owner's next call still waits.  Outputs
    are unchanged by the gating."""
    import ctypes
    import essential_matrix
    from sfm_amd import _lib, synth
    from sfm_amd.pipeline import TwoViewHotPath
    lib = _lib.load()
    B = 2
    flow, K, _, _ = synth.kitti_pair_batch(B, seed=6, device=cuda)
    owner = TwoViewHotPath(B, (376, 1242), (94, 311), 32, 8, device=cuda)
    other = TwoViewHotPath(B, (376, 1242), (94, 311), 32, 8, device=cuda)
    Kinv = owner.k_inverse(K)
    want = [t.clone() for t in owner.pose(flow, K, Kinv)]
    q = owner.pts[0, :, :2].contiguous(); qp = owner.pts[0, :, 2:].contiguous()
    E0, P0, n0 = essential_matrix.computeP(q, qp, 2000, 2000, 1, 1e-4)
    torch.cuda.synchronize()
    side = torch.cuda.Stream(device=cuda)
    own_s = torch.cuda.Stream(device=cuda)
    oth_s = torch.cuda.Stream(device=cuda)

    def timed(stream, fn):
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(stream):
            t0.record(stream)
            out = fn()
            t1.record(stream)
        t1.synchronize()
        return t0.elapsed_time(t1), out

    base, _ = timed(own_s, lambda: owner.pose(flow, K, Kinv))
    torch.cuda.synchronize()
    with torch.cuda.stream(side):
        torch.cuda._sleep(200_000_000)                       # ~0.1 s on the side stream
    assert lib.sfm_score_gate(ctypes.c_void_p(side.cuda_stream), ctypes.c_void_p(own_s.cuda_stream), 1) == 0
    # the other hot path and a plain computeP, each on its own stream: not held
    t_other, got_other = timed(oth_s, lambda: other.pose(flow, K, Kinv))
    assert t_other < base + 20.0, (base, t_other)
    t_cp, got_cp = timed(oth_s, lambda: essential_matrix.computeP(q, qp, 2000, 2000, 1, 1e-4))
    assert t_cp < base + 20.0, (base, t_cp)
    # the owner's next call is still held (the gate was not consumed by them)
    t_own, got_own = timed(own_s, lambda: owner.pose(flow, K, Kinv))
    assert t_own > base + 20.0, (base, t_own)
    torch.cuda.synchronize()
    for a, b_ in zip(want, got_own):
        assert torch.equal(a, b_)
    for a, b_ in zip(want, got_other):
        assert torch.equal(a, b_)
    assert torch.equal(got_cp[0], E0) and torch.equal(got_cp[1], P0) and got_cp[2] == n0
    # consumed: the owner's call after it runs free
    t_free, _ = timed(own_s, lambda: owner.pose(flow, K, Kinv))
    assert t_free < base + 20.0, (base, t_free)
