"""The bench's default step order: TwoViewHotPath.step_pipelined runs each
step's plane sweep on a side stream, overlapping the next step's pose stage.
Steps issued back to back (so the overlap really happens) must give the same
E, P, inlier counts and cost volume as plain sequential steps."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_pipelined_steps_equal_plain_steps(cuda):
    from sfm_amd import synth
    from sfm_amd.pipeline import TwoViewHotPath
    B, C, L, fhw = 2, 32, 32, (94, 311)
    steps = []
    for s in (11, 12, 13):
        flow, K, _, _ = synth.kitti_pair_batch(B, seed=s, device=cuda)
        ref, tgt = synth.features(B, C, *fhw, seed=s, device=cuda)
        steps.append((flow, K, ref, tgt))
    mk = lambda: TwoViewHotPath(B, (376, 1242), fhw, C, L, 2, 1e-4, 1.0, True, 0.6, device=cuda)
    plain, piped = mk(), mk()
    outs = [piped.step_pipelined(*a) for a in steps]      # back to back: sweep i overlaps pose i+1
    torch.cuda.synchronize()
    for a, o in zip(steps, outs):
        E, P, inl, _ = plain.step(*a)
        assert torch.equal(E, o[0]) and torch.equal(P, o[1]) and torch.equal(inl, o[2])
    torch.cuda.synchronize()
    assert torch.equal(plain.cost, piped.cost)            # the last step's volume
