"""The branch-matching machinery of the GPU gradient tests (tests/_parity.py), checked on the CPU: an fp32 run of
the oracle plays the implementation under test.  Its trace (per BatchNorm: the pre-activation, scale 1, shift 0) makes
the fp64 oracle follow the fp32 run's ReLU / MaxPool branches, and then the fp32 gradients agree with the fp64 ones to
fp32 rounding in EVERY tensor -- including siamese_t32-64's inc layers, where the kink pixels move the unmatched
fp64 gradient by 9e-3 (the reason the GPU tests match branches)."""
import torch

from _parity import branch_matched_reference, check_branch_matched, rel
from oracle import siamese_oracle as O
from oracle.golden import Fixture


def _fp32_run_with_trace(fx):
    P = {k: torch.from_numpy(v.copy()).requires_grad_(True) for k, v in fx.params0.items()}
    B = O.fresh_buffers(O.param_shapes(fx.model_type, fx.cfg))
    batch = fx.batch()
    O.RECORD = []
    try:
        out = O.forward(fx.model_type, P, B, batch['x_t1'], batch['x_t2'], fx.cfg, True)
        rec = O.RECORD
    finally:
        O.RECORD = None
    O.step_loss(fx.model_type, out, batch, fx.meta['alpha']).backward()
    names, trace = {}, []
    for key, z in rec:  # the BatchNorm output itself stands in for y (scale 1, shift 0)
        tag = object()
        names[id(tag)] = key
        trace.append((tag, z.permute(0, 2, 3, 1).contiguous(), torch.ones(z.shape[1]), torch.zeros(z.shape[1]), 1))
    return P, batch, {k: v.grad for k, v in P.items()}, trace, names, tag


def test_branch_matched_fp64_follows_the_fp32_run():
    fx = Fixture('siamese_t32-64')
    P, batch, g32, trace, names, _ = _fp32_run_with_trace(fx)
    loss = lambda out, bt: O.step_loss(fx.model_type, out, bt, fx.meta['alpha'])
    P0 = {k: v.detach() for k, v in P.items()}
    _, _, g64 = branch_matched_reference(fx.model_type, P0, batch, fx.cfg, trace, names, loss)
    order = list(P0)
    assert not check_branch_matched(g32, g64, order, 1e-4)
    # unmatched, the fp64 oracle takes its own branches at the kink pixels: a much larger difference somewhere
    Pd = {k: v.double().requires_grad_(True) for k, v in P0.items()}
    Bd = {k: (v.double() if v.is_floating_point() else v)
          for k, v in O.fresh_buffers(O.param_shapes(fx.model_type, fx.cfg)).items()}
    bd = {k: (v.double() if v.is_floating_point() else v) for k, v in batch.items()}
    loss(O.forward(fx.model_type, Pd, Bd, bd['x_t1'], bd['x_t2'], fx.cfg, True), bd).backward()
    worst_unmatched = max(rel(g32[k], Pd[k].grad) for k in order if not k.endswith(('conv.0.bias', 'conv.3.bias')))
    worst_matched = max(rel(g32[k], g64[k]) for k in order if not k.endswith(('conv.0.bias', 'conv.3.bias')))
    print(f'fp32 vs fp64 oracle gradients: unmatched {worst_unmatched:.2e}, branch-matched {worst_matched:.2e}')
    assert worst_matched < 1e-4 < worst_unmatched


def test_branch_match_rejects_a_foreign_trace():
    """A pre-activation that matches no traced one (here: another fixture's weights) is an error, not a silent
    fallback to the oracle's own branches."""
    fx = Fixture('siamese_t8-16')
    P, batch, _, trace, names, _ = _fp32_run_with_trace(fx)
    P2 = {k: (v.detach() * 1.5) for k, v in P.items()}
    loss = lambda out, bt: O.step_loss(fx.model_type, out, bt, fx.meta['alpha'])
    try:
        branch_matched_reference(fx.model_type, P2, batch, fx.cfg, trace, names, loss)
    except AssertionError as e:
        assert 'no GPU pre-activation' in str(e)
    else:
        raise AssertionError('a foreign trace was accepted')


def _bm_one(z_gpu):
    """A BranchMatch over one traced BatchNorm output whose GPU pre-activation is z_gpu (NCHW, scale 1, shift 0)."""
    from _parity import BranchMatch
    tag = object()
    c = z_gpu.shape[1]
    return BranchMatch([(tag, z_gpu.permute(0, 2, 3, 1).contiguous(), torch.ones(c), torch.zeros(c), 1)],
                       {id(tag): 'k'})


def test_branch_match_bounds_relu_flips():
    """A GPU ReLU decision against the oracle's own sign is adopted only inside the 1e-5 kink band: a flip at
    3e-6 of max is counted, one at 3e-5 of max (still within the 1e-4 distance guard) raises."""
    torch.manual_seed(0)
    z = torch.rand(1, 4, 6, 6) + 0.5
    z[0, 1, 2, 3] = 3e-6 * float(z.max())
    bm = _bm_one(torch.where(z.abs() < 1e-5 * z.max(), -z, z))
    m, _ = bm('k', z.double())
    assert bm.flips == 1 and not bool(m[0, 1, 2, 3])
    z[0, 1, 2, 3] = 3e-5 * float(z.max())
    bm = _bm_one(torch.where(z.abs() < 1e-4 * z.max(), -z, z))
    try:
        bm('k', z.double())
    except AssertionError as e:
        assert 'outside the kink band' in str(e)
    else:
        raise AssertionError('a ReLU flip outside the kink band was adopted')


def test_branch_match_bounds_pool_argmax():
    """A GPU pooling argmax that differs from the oracle's is adopted only at a near-tie."""
    z = torch.full((1, 1, 2, 2), 0.5)
    z[0, 0, 0, 0] = 1.0
    z[0, 0, 1, 1] = 1.0 - 4e-6
    g = z.clone()
    g[0, 0, 1, 1] = 1.0 + 4e-6  # within 1e-5 of max of the oracle's winner: a near-tie
    bm = _bm_one(g)
    bm('k', z.double())
    assert bm.pool_flips == 1 and bm.flips == 0
    z[0, 0, 1, 1] = 1.0 - 4e-5
    g[0, 0, 1, 1] = 1.0 + 4e-5  # distance 8e-5 < the 1e-4 guard, but a real argmax change
    try:
        _bm_one(g)('k', z.double())
    except AssertionError as e:
        assert 'near-tie' in str(e)
    else:
        raise AssertionError('a pooling argmax change outside the near-tie band was adopted')
