"""Model-level parity on MI355X: the HIP path vs golden fixtures produced by the reference itself.

Bars (north_star): logits within 1e-4 relative (max|d| / max|ref|) in fp32, change masks (logit > 0,
i.e. round(sigmoid) as utils/metrics.py:26) bit-exact outside the |logit_ref| < 1e-4*max band.
Gradients: 1e-3 relative per tensor against the fp64 oracle following the GPU forward's own ReLU / MaxPool
branches (tests/_parity.py branch matching), with no exemptions; the reference's fp32 gradients (which took their
own branches at kink-ambiguous pixels) within 2e-2 norm-wise.  Conv biases feeding a train-mode BatchNorm have a
true gradient of 0 and are checked for being ~0 instead.
"""
import numpy as np
import pytest
import torch

from _parity import branch_matched_reference, check_branch_matched, rel_l2
from oracle.golden import NAMES, Fixture, rel_err

pytestmark = pytest.mark.gpu

LOGIT_TOL = 1e-4
GRAD_TOL = 1e-3
FIXTURE_L2 = 2e-2


def _pre_bn_bias(k):
    return k.endswith('conv.0.bias') or k.endswith('conv.3.bias')


def kink_pixels(fx, rel=1e-6):
    """BN outputs z of the reference forward with |z| < rel * max|z|: there the ReLU mask (z > 0) depends on
    the last bit of z, so any fp32 reimplementation may route the gradient differently (one such pixel moved
    inc.conv.0.weight's gradient by 8e-3 in siamese_t8-16: z = 9.9e-9 vs scale ~3)."""
    from oracle import siamese_oracle as O
    P = {k: torch.from_numpy(v.copy()) for k, v in fx.params0.items()}
    B = O.fresh_buffers(O.param_shapes(fx.model_type, fx.cfg))
    batch = fx.batch()
    O.RECORD = []
    try:
        with torch.no_grad():
            O.forward(fx.model_type, P, B, batch['x_t1'], batch['x_t2'], fx.cfg, training=True)
        rec = O.RECORD
    finally:
        O.RECORD = None
    return [(k, float(z.abs().min())) for k, z in rec if float(z.abs().min()) < rel * float(z.abs().max())]


def _step_loss(model_type, alpha):
    from oracle import siamese_oracle as O
    return lambda out, batch: O.step_loss(model_type, out, batch, alpha)


def _build(fx, dev):
    from multimodal_siamese_cd_amd.utils import networks
    cfg = fx.package_cfg()
    net = networks.create_network(cfg)
    with torch.no_grad():
        for k, p in net.module.named_parameters():
            p.copy_(torch.from_numpy(fx.params0[k]))
    return cfg, net.to(dev)


def _outs(o):
    return list(o) if isinstance(o, (tuple, list)) else [o]


@pytest.fixture(scope='module')
def dev():
    from multimodal_siamese_cd_amd import hip
    hip.load_library()
    return torch.device('cuda:0')


def check_logits(out, ref):
    out = out.detach().cpu().numpy()
    assert out.shape == ref.shape
    assert rel_err(out, ref) < LOGIT_TOL
    band = np.abs(ref) < LOGIT_TOL * np.abs(ref).max()
    mism = ((out > 0) != (ref > 0)) & ~band
    assert not mism.any(), f'{mism.sum()} mask pixels differ outside the tolerance band'


@pytest.mark.parametrize('name', NAMES)
def test_train_step_matches_reference(dev, name):
    from multimodal_siamese_cd_amd import engine, trainers
    fx = Fixture(name)
    cfg, net = _build(fx, dev)
    net.train()
    batch = {k: v.to(dev) for k, v in fx.batch().items()}
    with engine.trace_bn() as trace:
        out = net(batch['x_t1'], batch['x_t2'])
    loss = trainers.step_loss(cfg, out, batch)
    loss.backward()
    for o, ref in zip(_outs(out), fx.outputs):
        check_logits(o, ref)
    assert abs(loss.item() - float(fx.z['loss0'])) < 1e-5
    grads = fx.grads
    bad, got = [], {}
    for k, p in net.module.named_parameters():
        if k not in grads:
            assert p.grad is None, k
            continue
        got[k] = p.grad.cpu()
        if _pre_bn_bias(k):
            g, w = got[k].numpy(), grads[k.replace('.bias', '.weight')]
            if not np.abs(g).max() < 1e-4 * max(np.abs(w).max(), 1e-3):
                bad.append((k, float(np.abs(g).max())))
    assert not bad, bad
    order = [k for k, _ in net.module.named_parameters() if k in grads]
    P = {k: torch.from_numpy(v.copy()) for k, v in fx.params0.items()}
    _, lref, ref = branch_matched_reference(fx.model_type, P, fx.batch(), fx.cfg, trace, net.module,
                                            _step_loss(fx.model_type, fx.meta['alpha']))
    assert abs(loss.item() - lref.item()) < 1e-5
    assert not check_branch_matched(got, ref, order, GRAD_TOL)
    l2 = {k: rel_l2(got[k], grads[k]) for k in order if not _pre_bn_bias(k)}
    worst = max(l2.items(), key=lambda kv: kv[1])
    print(f'gradients vs the reference fixture: worst rel-L2 {worst[1]:.2e} ({worst[0]})')
    assert worst[1] < FIXTURE_L2, worst
    r1 = fx.prefixed('r1/')
    sd = net.module.state_dict()
    for k, ref in r1.items():
        v = sd[k].cpu().numpy()
        if k.endswith('num_batches_tracked'):
            assert int(v) == int(ref), k
        else:
            assert rel_err(v, ref) < 1e-5, k


@pytest.mark.parametrize('name', NAMES)
def test_eval_forward_matches_reference(dev, name):
    from multimodal_siamese_cd_amd import trainers
    fx = Fixture(name)
    cfg, net = _build(fx, dev)
    net.train()
    batch = {k: v.to(dev) for k, v in fx.batch().items()}
    out = net(batch['x_t1'], batch['x_t2'])  # updates running statistics like the reference step did
    trainers.step_loss(cfg, out, batch).backward()
    net.eval()
    with torch.no_grad():
        ev = net(batch['x_t1'], batch['x_t2'])
    for o, ref in zip(_outs(ev), fx.eval_outputs):
        check_logits(o, ref)


@pytest.mark.parametrize('fused', [False, True])
@pytest.mark.parametrize('name', ['siamese_t8-16', 'siamese_t8-16-32', 'whatevernet_t8-16'])
def test_adamw_trajectory_matches_reference(dev, name, fused):
    """3 AdamW steps; fused=True is the bench's optimizer (it does not bump parameter versions, so any cache of
    derived weights must not key on them)."""
    from multimodal_siamese_cd_amd import trainers
    fx = Fixture(name)
    cfg, net = _build(fx, dev)
    opt = torch.optim.AdamW(net.parameters(), lr=fx.meta['lr'], weight_decay=fx.meta['wd'], fused=fused)
    batch = {k: v.to(dev) for k, v in fx.batch().items()}
    losses = []
    for _ in range(3):
        net.train()
        opt.zero_grad()
        loss = trainers.step_loss(cfg, net(batch['x_t1'], batch['x_t2']), batch)
        loss.backward()
        opt.step()
        losses.append(loss.item())
    np.testing.assert_allclose(losses, fx.z['losses'], atol=2e-5)
    p3 = fx.prefixed('p3/')
    kinks = None
    for k, p in net.module.named_parameters():
        if _pre_bn_bias(k):
            continue
        d = np.abs(p.detach().cpu().numpy() - p3[k])
        # Adam normalises each element: elements whose |g| is at fp32 noise level may step differently
        n_bad = int((d > 1e-5).sum())
        if n_bad > max(2, 1e-3 * d.size):
            kinks = kink_pixels(fx) if kinks is None else kinks
            assert kinks and float(d.max()) < 3 * fx.meta['lr'], (k, n_bad, d.size, kinks)


def test_siamese_bn_batches_are_per_branch(dev):
    """nseg=2: concatenating t1 and t2 into one BN batch would change outputs."""
    fx = Fixture('siamese_t8-16')
    cfg, net = _build(fx, dev)
    nbt = net.module.inc.conv.conv[1].num_batches_tracked.item()
    batch = {k: v.to(dev) for k, v in fx.batch().items()}
    net.train()
    with torch.no_grad():
        net(batch['x_t1'], batch['x_t2'])
    assert net.module.inc.conv.conv[1].num_batches_tracked.item() == nbt + 2  # encoder: t1 then t2
    assert net.module.decoder.up_seq.up1.conv.conv[1].num_batches_tracked.item() == 1


def test_state_dict_interchanges_with_reference_keys(dev):
    fx = Fixture('siamese_t8-16')
    _, net = _build(fx, dev)
    keys = set(net.state_dict())
    want = {'module.' + k for k in fx.params0} | {'module.' + k for k in fx.prefixed('r1/')}
    assert keys == want


def test_fused_input_bn_model_step(dev):
    """A topology whose DoubleConvs take the fused BN0 path (channels multiple of 32): fused and materialised
    runs are bit-identical, and both match the CPU oracle (logits, loss, gradients)."""
    from multimodal_siamese_cd_amd import engine, hip
    from multimodal_siamese_cd_amd.utils import experiment_manager, loss_functions, networks
    from oracle import siamese_oracle as O
    ocfg = dict(TOPOLOGY=[32, 64], IN_CHANNELS=5, OUT_CHANNELS=1, S1_BANDS=[0, 1], S2_BANDS=[2, 1, 0])
    shapes = O.param_shapes('siameseunet', ocfg)
    P = O.deterministic_params(shapes, 7)
    b = O.synthetic_batch(ocfg, 2, 64, 8)
    cfg = experiment_manager.new_config()
    cfg.MODEL.TYPE, cfg.MODEL.IN_CHANNELS, cfg.MODEL.OUT_CHANNELS = 'siameseunet', 5, 1
    cfg.MODEL.TOPOLOGY = [32, 64]
    cfg.DATALOADER.S1_BANDS, cfg.DATALOADER.S2_BANDS = [0, 1], [2, 1, 0]
    cfg.MODEL.CONV_MATH = 'x3'  # the fused/materialised comparison under the bound-free arithmetic
    crit = loss_functions.get_criterion('PowerJaccardLoss')
    runs, traces = [], []
    for fuse in (True, False):
        prev = engine.set_options(fuse_input_bn=fuse, fuse_bn_bwd=False)
        try:
            net = networks.create_network(cfg)
            with torch.no_grad():
                for k, p in net.module.named_parameters():
                    p.copy_(P[k])
            net.to(dev).train()
            with engine.trace_bn() as trace:
                out = net(b['x_t1'].to(dev), b['x_t2'].to(dev))
            loss = crit(out, b['y_change'].to(dev))
            loss.backward()
            runs.append((out.detach().cpu(), loss.item(),
                         {k: p.grad.detach().cpu() for k, p in net.module.named_parameters()}))
            traces.append((trace, net.module))
        finally:
            engine.set_options(**prev)
    (o1, l1, g1), (o0, l0, g0) = runs
    assert torch.equal(o1, o0) and l1 == l0
    for k in g1:
        assert torch.equal(g1[k], g0[k]), k
    # fused BatchNorm-backward partial sums: same result up to summation order
    prev = engine.set_options(fuse_input_bn=True, fuse_bn_bwd=True)
    try:
        net = networks.create_network(cfg)
        with torch.no_grad():
            for k, p in net.module.named_parameters():
                p.copy_(P[k])
        net.to(dev).train()
        loss = crit(net(b['x_t1'].to(dev), b['x_t2'].to(dev)), b['y_change'].to(dev))
        loss.backward()
        for k, p in net.module.named_parameters():
            if not _pre_bn_bias(k):
                assert rel_err(p.grad.cpu().numpy(), g1[k].numpy()) < 1e-4, k
    finally:
        engine.set_options(**prev)
    # against the CPU oracle: logits and loss vs fp32, gradients vs the fp64 oracle on the fused run's branches
    Pr = {k: v.clone() for k, v in P.items()}
    ref = O.forward('siameseunet', Pr, O.fresh_buffers(shapes), b['x_t1'], b['x_t2'], ocfg, True)
    lref = O.power_jaccard_loss(ref, b['y_change'])
    check_logits(o1, ref.detach().numpy())
    assert abs(l1 - lref.item()) < 1e-5
    _, _, gref = branch_matched_reference('siameseunet', P, b, ocfg, *traces[0], _step_loss('siameseunet', 0.5))
    assert not check_branch_matched(g1, gref, list(P), GRAD_TOL)


@pytest.mark.parametrize('name', ['siamese_t8-16', 'whatevernet_t8-16', 'siamese_t32-64'])
def test_fused_siamese_encoder_matches_unfused(dev, name):
    """SiameseLevelFn (BN + ReLU fused into pool / difference, zero-copy concat) vs the plain encoder +
    SiameseDiffFn path: logits bit-identical, gradients equal up to summation order."""
    from multimodal_siamese_cd_amd import engine, trainers
    fx = Fixture(name)
    res = []
    for fused in (True, False):
        prev = engine.set_options(fuse_siamese_encoder=fused)
        try:
            cfg, net = _build(fx, dev)
            net.train()
            batch = {k: v.to(dev) for k, v in fx.batch().items()}
            out = net(batch['x_t1'], batch['x_t2'])
            loss = trainers.step_loss(cfg, out, batch)
            loss.backward()
            res.append(([o.detach().cpu() for o in _outs(out)],
                        {k: p.grad.cpu() for k, p in net.module.named_parameters() if p.grad is not None}))
        finally:
            engine.set_options(**prev)
    for a, b in zip(res[0][0], res[1][0]):
        assert torch.equal(a, b)
    for k in res[0][1]:
        if not _pre_bn_bias(k):
            assert rel_err(res[0][1][k].numpy(), res[1][1][k].numpy()) < 1e-5, k


@pytest.mark.parametrize('name', ['siamese_t8-16', 'siamese_t8-16-32_odd', 'unet_t8-16', 'dtsiamese_t8-16',
                                  'siamese_t32-64', 'dtsiamese_t32-64'])  # the last two under h2 (32/64 channels)
def test_fused_head_bit_identical(dev, name):
    """The 1x1 head fused into the decoder stage (engine fuse_head: forward through the last BatchNorm's
    coefficients, backward through scd_bn_relu_backward_head) vs the materialised decoder output + HeadFn:
    logits, loss and every gradient bit-identical, in train and eval mode."""
    from multimodal_siamese_cd_amd import engine, trainers
    fx = Fixture(name)
    res = []
    for fused in (True, False):
        prev = engine.set_options(fuse_head=fused, head_wgrad_in_bn_bwd=False)
        try:
            cfg, net = _build(fx, dev)
            net.train()
            batch = {k: v.to(dev) for k, v in fx.batch().items()}
            out = net(batch['x_t1'], batch['x_t2'])
            loss = trainers.step_loss(cfg, out, batch)
            loss.backward()
            net.eval()
            with torch.no_grad():
                ev = net(batch['x_t1'], batch['x_t2'])
            res.append(([o.detach().cpu() for o in _outs(out)], loss.item(), [o.cpu() for o in _outs(ev)],
                        {k: p.grad.cpu() for k, p in net.module.named_parameters() if p.grad is not None}))
        finally:
            engine.set_options(**prev)
    (o1, l1, e1, g1), (o0, l0, e0, g0) = res
    assert l1 == l0
    for a, b in zip(o1 + e1, o0 + e0):
        assert torch.equal(a, b)
    assert g1.keys() == g0.keys()
    for k in g0:
        assert torch.equal(g1[k], g0[k]), k


@pytest.mark.parametrize('name', ['siamese_t8-16', 'siamese_t8-16-32_odd', 'dtsiamese_t8-16'])
def test_head_weight_grad_from_bn_backward(dev, name):
    """The fused head's weight grad taken in its BatchNorm's partial pass (engine head_wgrad_in_bn_bwd:
    scd_bn_relu_backward_head w_grad) vs its own weighted channel sum (scd_conv1x1_bwd_bn gw): logits, loss and every
    other gradient bit-identical, the head weights' within 1e-6 (same chunks and tree, the products' rounding may
    contract differently)."""
    from multimodal_siamese_cd_amd import engine, trainers
    fx = Fixture(name)
    res = []
    for fold in (True, False):
        prev = engine.set_options(fuse_head=True, head_wgrad_in_bn_bwd=fold)
        try:
            cfg, net = _build(fx, dev)
            net.train()
            batch = {k: v.to(dev) for k, v in fx.batch().items()}
            out = net(batch['x_t1'], batch['x_t2'])
            loss = trainers.step_loss(cfg, out, batch)
            loss.backward()
            res.append(([o.detach().cpu() for o in _outs(out)], loss.item(),
                        {k: p.grad.cpu() for k, p in net.module.named_parameters() if p.grad is not None}))
        finally:
            engine.set_options(**prev)
    (o1, l1, g1), (o0, l0, g0) = res
    assert l1 == l0
    for a, b in zip(o1, o0):
        assert torch.equal(a, b)
    assert g1.keys() == g0.keys()
    heads = [k for k in g0 if k.startswith('outc') and k.endswith('weight')]
    assert heads
    for k in g0:
        if k in heads:
            assert ((g1[k] - g0[k]).abs().max() / g0[k].abs().max()).item() < 1e-6, k
        else:
            assert torch.equal(g1[k], g0[k]), k


@pytest.mark.parametrize('name', ['siamese_t8-16', 'siamese_t8-16-32_odd', 'whatevernet_t8-16'])
def test_pooled_bn_backward_matches_unfused(dev, name):
    """The encoder BatchNorm backward forming maxpool_bwd -/+ the difference gradient on the fly over Siamese pairs
    (scd_bn_relu_backward_pooled) vs materialising it (scd_feature_grad, then scd_bn_relu_backward): every gradient
    up to the order of the BatchNorm partial sums."""
    from multimodal_siamese_cd_amd import engine, trainers
    fx = Fixture(name)
    res = []
    for pooled in (True, False):
        prev = engine.set_options(pooled_bn_bwd=pooled)
        try:
            cfg, net = _build(fx, dev)
            net.train()
            batch = {k: v.to(dev) for k, v in fx.batch().items()}
            loss = trainers.step_loss(cfg, net(batch['x_t1'], batch['x_t2']), batch)
            loss.backward()
        finally:
            engine.set_options(**prev)
        res.append({k: p.grad.cpu() for k, p in net.module.named_parameters() if p.grad is not None})
    for k in res[1]:  # the pooled walk sums its partials over 2x2 cells: equal up to summation order
        if not _pre_bn_bias(k):
            assert rel_err(res[0][k].numpy(), res[1][k].numpy()) < 1e-5, k


@pytest.mark.parametrize('name', ['siamese_t32-64', 'dtsiamese_t32-64', 'dualstream_t32-64'])
def test_reference_fixtures_reach_the_h2_kernels(dev, monkeypatch, name):
    """The 32/64-channel reference fixtures run on the production kernels: built through create_network (MODEL.
    PRECISION fp32 -> h2), every conv launch runs the arithmetic it would with bounds on all operands, and the 3x3
    convs with 32-channel-multiple sources and >= 64 outputs run h2."""
    from _parity import record_arith
    from multimodal_siamese_cd_amd import trainers
    fx = Fixture(name)
    cfg, net = _build(fx, dev)
    assert net.module.conv_math == 'h2'
    net.train()
    batch = {k: v.to(dev) for k, v in fx.batch().items()}
    seen = record_arith(monkeypatch, dev)
    trainers.step_loss(cfg, net(batch['x_t1'], batch['x_t2']), batch).backward()
    monkeypatch.undo()
    assert all(s[4] == s[5] for s in seen), [s for s in seen if s[4] != s[5]]
    # the h2 halo kernels tile >= 64 output channels: every such 3x3 conv with a 32-channel-multiple source runs h2
    h2 = [s for s in seen if s[3] == 9 and s[1] % 32 == 0 and s[2] % 64 == 0]
    assert h2 and all(s[4] == 'h2' for s in h2), [s for s in h2 if s[4] != 'h2']
    print(f'{sum(s[4] == "h2" for s in seen)} of {len(seen)} conv launches run h2')


def test_padded_twin_survives_a_device_change(dev):
    """A TOPOLOGY off the channel granule (here [12, 20]) runs a zero-padded twin whose parameters are plain attributes
    after the first build; moving the twin to another device and back rebuilds only the index maps (the parameter
    shapes are kept from the first build) and the forward gives the same logits."""
    from multimodal_siamese_cd_amd.utils import experiment_manager as em, networks
    cfg = em.load_cfg('debug')
    cfg.MODEL.TOPOLOGY = [12, 20]
    torch.manual_seed(0)
    net = networks.create_network(cfg).to(dev).eval()
    g = torch.Generator(device=dev).manual_seed(2)
    x1 = torch.rand(2, 5, 32, 32, device=dev, generator=g)
    x2 = torch.rand(2, 5, 32, 32, device=dev, generator=g)
    with torch.no_grad():
        out0 = net(x1, x2).clone()
        net.module._twin_ready(torch.device('cpu'))  # the twin moves away: maps rebuilt without its parameters
        out1 = net(x1, x2)  # and back to the GPU
    assert torch.equal(out0, out1)
