"""The building blocks called on their own (NCHW in, NCHW out, autograd), as the reference's callers use them:
Encoder, Decoder, DoubleConv, InConv, Down, Up, OutConv (utils/networks.py:313-461) and the direct head call
net.module.outc_sem_change(torch.cat((s1, s2), 1)) of assessment_semantics.py:34,117.

Each block runs on the HIP kernels in the model's arithmetic (h2 here, channels that take the h2 kernels) against
the CPU oracle's functional restatement of the same block in fp64: outputs within 1e-4 relative, input and
parameter gradients within 1e-3, BatchNorm running statistics within 1e-5.  Parameters come from the
reference-generated dtsiamese_t32-64 fixture.
"""
import pytest
import torch
import torch.nn.functional as F

from _parity import rel
from oracle.golden import Fixture

pytestmark = pytest.mark.gpu

OUT_TOL = 1e-4
GRAD_TOL = 1e-3


@pytest.fixture(scope='module')
def dev():
    from multimodal_siamese_cd_amd import hip
    hip.load_library()
    return torch.device('cuda:0')


@pytest.fixture
def net(dev):
    from multimodal_siamese_cd_amd.utils import networks
    fx = Fixture('dtsiamese_t32-64')
    n = networks.create_network(fx.package_cfg())
    with torch.no_grad():
        for k, p in n.module.named_parameters():
            p.copy_(torch.from_numpy(fx.params0[k]))
    return n.to(dev).train()


def _params(module, prefix=''):
    return {prefix + k: p.detach().cpu().double().clone().requires_grad_(True) for k, p in module.named_parameters()}


def _buffers(module, prefix=''):
    return {prefix + k: (v.detach().cpu().double().clone() if v.is_floating_point() else v.detach().cpu().clone())
            for k, v in module.named_buffers()}


def _rand(shape, seed, grad=True):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(shape, generator=g).requires_grad_(grad)


def _run(block, inputs, dev, seed, training=True):
    """Forward on the GPU (model arithmetic), backward of sum(out * G); returns out, input grads, param grads."""
    from multimodal_siamese_cd_amd import hip
    block.train(training)
    xs = [x.detach().to(dev).requires_grad_(x.requires_grad) for x in inputs]
    with hip.conv_scope('h2'):
        out = block(*xs)
        outs = out if isinstance(out, list) else [out]
        gs = [_rand(o.shape, seed + i, False).to(dev) for i, o in enumerate(outs)]
        if training:
            sum((o * g).sum() for o, g in zip(outs, gs)).backward()
    torch.cuda.synchronize()
    return ([o.detach().cpu() for o in outs], [None if x.grad is None else x.grad.cpu() for x in xs],
            {k: p.grad.cpu() for k, p in block.named_parameters() if p.grad is not None}, [g.cpu() for g in gs])


def _ref_backward(outs, gs, inputs, P):
    for x in inputs:
        if x.grad is not None:
            x.grad = None
    sum((o * g.double()).sum() for o, g in zip(outs, gs)).backward()
    return [None if x.grad is None else x.grad for x in inputs], {k: v.grad for k, v in P.items()}


def _check(got, ref_outs, ref_in_grads, ref_pgrads, block, buffers_ref=None):
    outs, in_grads, pgrads, _ = got
    for o, r in zip(outs, ref_outs):
        assert o.shape == r.shape
        assert rel(o, r) < OUT_TOL, rel(o, r)
    for g, r in zip(in_grads, ref_in_grads):
        if r is not None:
            assert g is not None and rel(g, r) < GRAD_TOL, rel(g, r)
    for k, r in ref_pgrads.items():
        if k.endswith('conv.0.bias') or k.endswith('conv.3.bias'):  # pre-BatchNorm biases: true gradient 0, float
            # noise of a sum over every pixel; judged against the same conv's weight gradient
            wk = k[:-len('bias')] + 'weight'
            assert pgrads[k].abs().max() < 1e-3 * ref_pgrads[wk].abs().max().item(), k
            continue
        assert rel(pgrads[k], r) < GRAD_TOL, (k, rel(pgrads[k], r))
    if buffers_ref is not None:
        sd = {k: v.cpu() for k, v in block.named_buffers()}
        for k, v in buffers_ref.items():
            if k.endswith('running_mean') or k.endswith('running_var'):
                assert rel(sd[k], v) < 1e-5, k
            else:
                assert int(sd[k]) == int(v), k


def test_double_conv_and_inconv(dev, net):
    from oracle import siamese_oracle as O
    inc = net.module.inc
    x = _rand((2, 32, 40, 24), 1)  # a 32-channel source (takes the h2 halo kernels), odd-ish map
    dc = net.module.encoder.down_seq.down1.mpconv[1]  # DoubleConv(32, 64)
    P, B = _params(dc), _buffers(dc)
    got = _run(dc, [x], dev, 10)
    xr = x.detach().double().requires_grad_(True)
    ref = O.double_conv(xr, P, B, '', True)
    rin, rp = _ref_backward([ref], got[3], [xr], P)
    _check(got, [ref.detach()], rin, rp, dc, B)
    # InConv: the 5-band input layer (channels zero-padded to the 16-channel kernels; no input gradient there)
    x5 = _rand((2, 5, 32, 48), 2, grad=False)
    P, B = _params(inc), _buffers(inc)
    got = _run(inc, [x5], dev, 20)
    ref = O.double_conv(x5.double(), P, B, 'conv.', True)
    rin, rp = _ref_backward([ref], got[3], [x5], P)
    _check(got, [ref.detach()], rin, rp, inc, B)


def test_double_conv_eval_mode(dev, net):
    from oracle import siamese_oracle as O
    dc = net.module.decoder_sem.up_seq.up1.conv  # DoubleConv(64, 32)
    g = torch.Generator().manual_seed(5)
    with torch.no_grad():
        for bn in (dc.conv[1], dc.conv[4]):
            bn.running_mean.copy_(torch.randn(bn.num_features, generator=g) * 0.1)
            bn.running_var.copy_(torch.rand(bn.num_features, generator=g) + 0.5)
    x = _rand((2, 64, 32, 32), 3, grad=False)
    P, B = _params(dc), _buffers(dc)
    got = _run(dc, [x], dev, 30, training=False)
    ref = O.double_conv(x.double(), P, B, '', False)
    assert rel(got[0][0], ref) < OUT_TOL


def test_down(dev, net):
    from oracle import siamese_oracle as O
    down = net.module.encoder.down_seq.down2  # MaxPool2d(2) + DoubleConv(64, 64)
    x = _rand((2, 64, 34, 30), 4)  # even sizes; MaxPool floors
    P, B = _params(down), _buffers(down)
    got = _run(down, [x], dev, 40)
    xr = x.detach().double().requires_grad_(True)
    ref = O.double_conv(F.max_pool2d(xr, 2), P, B, 'mpconv.1.', True)
    rin, rp = _ref_backward([ref], got[3], [xr], P)
    _check(got, [ref.detach()], rin, rp, down, B)


@pytest.mark.parametrize('hw2', [(32, 32), (33, 35)])  # power-of-two and F.pad sizes (networks.py:440-443)
def test_up(dev, net, hw2):
    from oracle import siamese_oracle as O
    up = net.module.decoder_change.up_seq.up1  # ConvT(32, 32) -> cat(skip 32, up 32) -> DoubleConv(64, 32)
    x1 = _rand((2, 32, 16, 16), 5)
    x2 = _rand((2, 32) + hw2, 6)
    P, B = _params(up), _buffers(up)
    got = _run(up, [x1, x2], dev, 50)
    x1r, x2r = x1.detach().double().requires_grad_(True), x2.detach().double().requires_grad_(True)
    ref = O.up(x1r, x2r, P, B, '', True)
    rin, rp = _ref_backward([ref], got[3], [x1r, x2r], P)
    _check(got, [ref.detach()], rin, rp, up, B)


def test_encoder_and_decoder(dev, net):
    """Encoder.forward returns [x, down1(x), ...] reversed (networks.py:334-343); Decoder.forward pops the deepest
    map off its argument and runs the Up blocks (375-382)."""
    from oracle import siamese_oracle as O
    enc, dec = net.module.encoder, net.module.decoder_change
    topo = list(net.module.cfg.MODEL.TOPOLOGY)
    x = _rand((2, 32, 32, 32), 7)
    P = {**_params(enc, 'encoder.'), **_params(dec, 'decoder_change.')}
    B = {**_buffers(enc, 'encoder.'), **_buffers(dec, 'decoder_change.')}
    from multimodal_siamese_cd_amd import hip
    xd = x.detach().to(dev).requires_grad_(True)
    with hip.conv_scope('h2'):
        feats = enc(xd)
        assert len(feats) == len(topo) + 1 and feats[-1] is xd
        lst = list(feats)
        out = dec(lst)
        assert len(lst) == len(topo)  # popped, as the reference's Decoder does to its caller's list
        gout = _rand(out.shape, 70, False).to(dev)
        (out * gout).sum().backward()
    xr = x.detach().double().requires_grad_(True)
    rfeats = [xr]
    for i in range(len(topo)):
        rfeats.append(O.double_conv(F.max_pool2d(rfeats[-1], 2), P, B, f'encoder.down_seq.down{i + 1}.mpconv.1.', True))
    rfeats = rfeats[::-1]
    for f, r in zip(feats, rfeats):
        assert rel(f.detach(), r.detach()) < OUT_TOL
    rout = O.decoder(rfeats, P, B, 'decoder_change.', topo, True)
    assert rel(out.detach(), rout.detach()) < OUT_TOL
    (rout * gout.cpu().double()).sum().backward()
    assert rel(xd.grad, xr.grad) < GRAD_TOL
    for name, mod in (('encoder.', enc), ('decoder_change.', dec)):
        for k, p in mod.named_parameters():
            if k.endswith('conv.0.bias') or k.endswith('conv.3.bias'):
                continue
            assert rel(p.grad, P[name + k].grad) < GRAD_TOL, k


def test_outc_sem_change_direct_call(dev, net):
    """net.module.outc_sem_change(torch.cat((s1, s2), 1)) (assessment_semantics.py:34,117): a 2 -> 1 channel 1x1
    conv on NCHW logits, with gradients."""
    s1, s2 = _rand((2, 1, 64, 48), 8), _rand((2, 1, 64, 48), 9)
    head = net.module.outc_sem_change
    got = _run(head, [torch.cat((s1, s2), 1).detach().requires_grad_(True)], dev, 80)
    W, b = head.conv.weight.detach().cpu().double().requires_grad_(True), head.conv.bias.detach().cpu().double()
    b = b.requires_grad_(True)
    xr = torch.cat((s1, s2), 1).detach().double().requires_grad_(True)
    ref = F.conv2d(xr, W, b)
    (ref * got[3][0].double()).sum().backward()
    assert rel(got[0][0], ref.detach()) < 1e-6
    assert rel(got[1][0], xr.grad) < 1e-6
    assert rel(got[2]['conv.weight'], W.grad) < 1e-5 and rel(got[2]['conv.bias'], b.grad) < 1e-5


def test_out_conv_wide_head(dev):
    """OutConv with more than 4 outputs and a source of 6 channels: groups of 4 outputs on the 1x1 kernel, the source
    zero-padded to a multiple of 4 (the reference builds any OUT_CHANNELS)."""
    from multimodal_siamese_cd_amd.utils import networks
    torch.manual_seed(3)
    head = networks.OutConv(6, 7).to(dev)
    x = _rand((2, 6, 16, 24), 11)
    got = _run(head, [x], dev, 90)
    W = head.conv.weight.detach().cpu().double().requires_grad_(True)
    b = head.conv.bias.detach().cpu().double().requires_grad_(True)
    xr = x.detach().double().requires_grad_(True)
    ref = F.conv2d(xr, W, b)
    (ref * got[3][0].double()).sum().backward()
    assert got[0][0].shape == (2, 7, 16, 24)
    assert rel(got[0][0], ref.detach()) < 1e-6
    assert rel(got[1][0], xr.grad) < 1e-6
    assert rel(got[2]['conv.weight'], W.grad) < 1e-5 and rel(got[2]['conv.bias'], b.grad) < 1e-5
