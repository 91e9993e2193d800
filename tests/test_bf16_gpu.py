"""bf16 conv arithmetic (SCD_MATH_BF16; BASELINE configs baseline_dualstream / siamese_mmcr: dtype bf16).

Kernel level: the 16x16x32 halo kernels in bf16 mode compute an fp32-accumulated GEMM of bf16-rounded (RNE)
operands, so they are checked against torch fp32 convs of the *bf16-rounded* operands at the fp32 tolerance
(1e-5), and shown to differ from the exact fp32 result by a bf16-sized amount (the mode is really active).
Model level: a TOPOLOGY [64, 128] SiameseUNet (channel counts the bf16 kernels take) against the fp32 oracle at
bf16 tolerances (see test_bf16_siamese_model_step).
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from _parity import _CONVT2D, convT_bf16

TOL = 1e-5
_CONV2D = F.conv2d  # unpatched (the model test swaps F.conv2d inside the oracle run)


@pytest.fixture(scope='module')
def dev():
    from multimodal_siamese_cd_amd import hip
    hip.load_library()
    d = torch.device('cuda:0')
    hip.ensure_device(torch.empty(1, device=d))
    return d


@pytest.fixture
def bf16(dev):
    from multimodal_siamese_cd_amd import hip
    prev = hip.set_conv_math('bf16')
    yield
    hip.set_conv_math(prev)


def rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


def r16(t):
    return t.to(torch.bfloat16).float()


def nchw(t):
    return t.permute(0, 3, 1, 2).contiguous()


def nhwc_t(t):
    return t.permute(0, 2, 3, 1).contiguous()


SHAPES = [(2, 16, 32, 64, 128), (2, 16, 16, 128, 64), (1, 16, 16, 512, 512), (4, 8, 16, 64, 64), (2, 32, 32, 256, 256)]


@pytest.mark.parametrize('n,h,w,ci,co', SHAPES)
def test_bf16_conv_forward_and_data_grad(dev, bf16, n, h, w, ci, co):
    from multimodal_siamese_cd_amd import hip
    g = torch.Generator().manual_seed(n + h + ci + co)
    x = torch.randn(n, h, w, ci, generator=g)
    wt = torch.randn(co, ci, 3, 3, generator=g) / (3 * ci ** 0.5)
    b = torch.randn(co, generator=g)
    wd = wt.to(dev)
    y = torch.empty(n, h, w, co, device=dev)
    hip.conv_igemm(hip.nhwc(x.to(dev)), h, w, 1, hip.TAPS_3X3, hip.pack_conv3x3(wd, 0), co, b.to(dev), hip.nhwc(y))
    ref16 = nhwc_t(F.conv2d(nchw(r16(x)).double(), r16(wt).double(), b.double(), padding=1))
    ref32 = nhwc_t(F.conv2d(nchw(x).double(), wt.double(), b.double(), padding=1))
    assert rel(y, ref16) < TOL
    assert rel(y, ref32) > 1e-4  # bf16 operands really used
    dy = torch.randn(n, h, w, co, generator=g)
    dx = torch.empty(n, h, w, ci, device=dev)
    hip.conv_igemm(hip.nhwc(dy.to(dev)), h, w, 1, hip.TAPS_3X3, hip.pack_conv3x3(wd, 1), ci, None, hip.nhwc(dx))
    ref_dx = nhwc_t(torch.nn.grad.conv2d_input((n, ci, h, w), r16(wt).double(), nchw(r16(dy)).double(), padding=1))
    assert rel(dx, ref_dx) < TOL


@pytest.mark.parametrize('n,h,w,ci,co', [(2, 8, 8, 64, 64), (3, 5, 7, 128, 64), (8, 64, 64, 64, 64),
                                         (2, 16, 16, 256, 128), (1, 4, 4, 512, 512)])
def test_bf16_convT_gather16(dev, bf16, n, h, w, ci, co):
    """The ConvTranspose forward (1 tap, pixel-shuffle store into a concat slice) and data grad (4 taps, stride-2
    gather from a channel slice) take the gather kernel's bf16 instance (no bound needed): fp32-accurate against
    the ConvT of the bf16-rounded operands, a bf16-sized distance from the exact result; the weight grad likewise on
    the generic weight grad's bf16 instance."""
    from multimodal_siamese_cd_amd import hip
    g = torch.Generator().manual_seed(n * h * w + ci + 1)
    x = torch.randn(n, h, w, ci, generator=g)
    wt = torch.randn(ci, co, 2, 2, generator=g) / 8
    b = torch.randn(co, generator=g)
    wf, wb = hip.pack_convT2x2(wt.to(dev), 0), hip.pack_convT2x2(wt.to(dev), 1)
    xd = x.to(dev)
    cat = torch.zeros(n, 2 * h, 2 * w, co + 32, device=dev)
    assert hip.igemm_arith(hip.nhwc(xd), h, w, 1, hip.TAPS_1, wf, 4 * co, hip.nhwc(cat, 32, co), store_mode=1) == 'bf16'
    hip.conv_igemm(hip.nhwc(xd), h, w, 1, hip.TAPS_1, wf, 4 * co, b.to(dev), hip.nhwc(cat, 32, co), store_mode=1)
    up = nchw(cat[..., 32:])
    ref16 = _CONVT2D(nchw(r16(x)).double(), r16(wt).double(), b.double(), stride=2)
    ref32 = _CONVT2D(nchw(x).double(), wt.double(), b.double(), stride=2)
    assert rel(up, ref16) < TOL
    assert rel(up, ref32) > 1e-4  # bf16 operands really used
    assert torch.equal(cat[..., :32], torch.zeros_like(cat[..., :32]))
    gcat = torch.randn(n, 2 * h, 2 * w, co + 32, generator=g)
    gcd = gcat.to(dev)
    assert hip.igemm_arith(hip.nhwc(gcd, 32, co), h, w, 2, hip.TAPS_2X2, wb, ci, hip.nhwc(xd)) == 'bf16'
    gx = torch.empty(n, h, w, ci, device=dev)
    hip.conv_igemm(hip.nhwc(gcd, 32, co), h, w, 2, hip.TAPS_2X2, wb, ci, None, hip.nhwc(gx))
    ref_gx = _CONV2D(nchw(r16(gcat[..., 32:])).double(), r16(wt).double(), None, stride=2)
    assert rel(nchw(gx), ref_gx) < TOL
    # weight grad: rows = the ConvT input, src = g_up gathered with stride 2 -> the generic weight grad's bf16 instance
    d, nsplit, nbytes = hip.wgrad_plan(hip.nhwc(xd), hip.nhwc(gcd, 32, co), 2, hip.TAPS_2X2)
    assert hip.wgrad_arith(d) == 'bf16'
    slabs = torch.empty(nbytes // 4, device=dev)
    hip.conv_wgrad(d, slabs)
    gw = torch.empty(ci, co, 2, 2, device=dev)
    hip.wgrad_finalize(slabs, nsplit, ci, 4, co, 1, co, gw)
    xr = nchw(r16(x)).double()
    wr = wt.double().requires_grad_(True)
    _CONVT2D(xr, wr, None, stride=2).backward(nchw(r16(gcat[..., 32:])).double())
    assert rel(gw, wr.grad) < TOL
    # the emulation the model-level oracles use agrees with the kernels
    xr = nchw(x).requires_grad_(True)
    wr = wt.clone().requires_grad_(True)
    y = convT_bf16(xr, wr, b, stride=2)
    assert rel(up, y.detach()) < TOL
    y.backward(nchw(gcat[..., 32:]))
    assert rel(nchw(gx), xr.grad) < TOL
    assert rel(gw, wr.grad) < TOL


@pytest.mark.parametrize('n,h,w,ci,co', SHAPES)
def test_bf16_conv_weight_grad(dev, bf16, n, h, w, ci, co):
    from multimodal_siamese_cd_amd import hip
    g = torch.Generator().manual_seed(3 * n + w + ci + co)
    x = torch.randn(n, h, w, ci, generator=g)
    dy = torch.randn(n, h, w, co, generator=g)
    d, nsplit, nbytes = hip.wgrad_plan(hip.nhwc(dy.to(dev)), hip.nhwc(x.to(dev)), 1, hip.TAPS_3X3)
    slabs = torch.empty(nbytes // 4, device=dev)
    hip.conv_wgrad(d, slabs)
    dw = torch.empty(co, ci, 3, 3, device=dev)
    hip.wgrad_finalize(slabs, nsplit, co, 9, ci, 0, ci, dw)
    ref16 = torch.nn.grad.conv2d_weight(nchw(r16(x)).double(), (co, ci, 3, 3), nchw(r16(dy)).double(), padding=1)
    ref32 = torch.nn.grad.conv2d_weight(nchw(x).double(), (co, ci, 3, 3), nchw(dy).double(), padding=1)
    assert rel(dw, ref16) < TOL
    assert rel(dw, ref32) > 1e-4


def test_bf16_fused_input_bn_is_bit_identical(dev, bf16):
    """In bf16 mode the BN-apply + ReLU fused into the halo staging still equals the materialised activation."""
    from multimodal_siamese_cd_amd import hip
    n, h, w, ci, co, nseg = 4, 16, 32, 64, 128, 2
    g = torch.Generator().manual_seed(11)
    y = torch.randn(n, h, w, ci, generator=g).to(dev)
    sc = (torch.rand(nseg * ci, generator=g) * 2 - 0.5).to(dev)
    sh = torch.randn(nseg * ci, generator=g).to(dev)
    a = torch.empty_like(y)
    hip.bn_relu_apply(hip.nhwc(y), nseg, sc, sh, hip.nhwc(a))
    wpk = hip.pack_conv3x3((torch.randn(co, ci, 3, 3, generator=g) / 24).to(dev), 0)
    o1, o2 = torch.empty(n, h, w, co, device=dev), torch.empty(n, h, w, co, device=dev)
    hip.conv_igemm(hip.nhwc(a), h, w, 1, hip.TAPS_3X3, wpk, co, None, hip.nhwc(o1))
    hip.conv_igemm(hip.nhwc(y), h, w, 1, hip.TAPS_3X3, wpk, co, None, hip.nhwc(o2), in_bn=(sc, sh, nseg))
    assert torch.equal(o1, o2)


class _Conv16(torch.autograd.Function):
    """A 3x3 conv with the bf16 kernels' arithmetic: bf16-rounded operands in forward, data-grad and weight-grad,
    exact products, fp32 (here double) accumulation."""

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        return _CONV2D(r16(x).double(), r16(w).double(), None, padding=1).float() + b[None, :, None, None]

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        g16 = r16(gy).double()
        gx = torch.nn.grad.conv2d_input(x.shape, r16(w).double(), g16, padding=1).float()
        gw = torch.nn.grad.conv2d_weight(r16(x).double(), w.shape, g16, padding=1).float()
        return gx, gw, gy.sum((0, 2, 3))


def _oracle_step(P, B, batch, ocfg, bf16_convs: bool):
    """The fp32 oracle's train step; with bf16_convs every 3x3 conv the bf16 kernels take (input channels a
    multiple of 32, or the input layer's bands, zero-padded to the 16-channel kernels: every 3x3 conv at
    TOPOLOGY [64, 128]) runs through _Conv16."""
    from oracle import siamese_oracle as O
    def conv(x, w, b=None, stride=1, padding=0, *a, **k):
        if (bf16_convs and w.shape[2:] == (3, 3) and (w.shape[1] % 32 == 0 or w.shape[1] <= 16) and stride == 1
                and padding == 1):
            return _Conv16.apply(x, w, b)
        return _CONV2D(x, w, b, stride, padding, *a, **k)

    P = {k: v.detach().clone().requires_grad_(True) for k, v in P.items()}
    B = {k: v.clone() for k, v in B.items()}
    F.conv2d = conv
    if bf16_convs:
        F.conv_transpose2d = convT_bf16  # the ConvTranspose forward / data grad on the bf16 gather kernel
    try:
        out = O.forward('siameseunet', P, B, batch['x_t1'], batch['x_t2'], ocfg, True)
        loss = O.power_jaccard_loss(out, batch['y_change'])
        loss.backward()
    finally:
        F.conv2d = _CONV2D
        F.conv_transpose2d = _CONVT2D
    return out.detach(), loss.detach(), {k: v.grad for k, v in P.items()}


def test_bf16_siamese_model_step(dev):
    """Train step of a TOPOLOGY [64, 128] SiameseUNet (64x64 tiles: every level takes the bf16 halo kernels).

    bf16 roundings amplify through depth (an fp32-level difference flips an occasional bf16 rounding, whose
    0.4% error then flips more in the next layer), so no implementation matches another bf16 implementation
    to fp32 precision at model level; the per-kernel tests above pin the arithmetic exactly.  Here:
      - logits within 3e-2 relative of the fp32 oracle, loss within 1e-2;
      - the logits closer to the oracle with the bf16 arithmetic emulated in its convs than to the plain fp32
        oracle (the bf16 semantics, not some other error);
      - every weight gradient with cosine similarity > 0.95 to the fp32 one (the emulated oracle itself
        reaches 0.975 at worst on this case)."""
    from multimodal_siamese_cd_amd import hip
    from multimodal_siamese_cd_amd.utils import experiment_manager as em, loss_functions, networks
    from oracle import siamese_oracle as O
    cfg = em.load_cfg('debug')
    ocfg = dict(TYPE='siameseunet', TOPOLOGY=[64, 128], IN_CHANNELS=5, OUT_CHANNELS=1, S1_BANDS=[0, 1],
                S2_BANDS=[2, 1, 0])
    shapes = O.param_shapes('siameseunet', ocfg)
    P = O.deterministic_params(shapes, 3)
    B = O.fresh_buffers(shapes)
    batch = O.synthetic_batch(ocfg, 2, 64, 4)
    out32, loss32, g32 = _oracle_step(P, B, batch, ocfg, False)
    out16, loss16, _ = _oracle_step(P, B, batch, ocfg, True)
    cfg.MODEL.PRECISION = 'bf16'  # create_network gives the model the bf16 arithmetic
    net = networks.create_network(cfg).to(dev)
    assert net.module.conv_math == 'bf16'
    with torch.no_grad():
        for k, p in net.module.named_parameters():
            p.copy_(P[k])
    net.train()
    out = net(batch['x_t1'].to(dev), batch['x_t2'].to(dev))
    loss = loss_functions.get_criterion('PowerJaccardLoss')(out, batch['y_change'].to(dev))
    loss.backward()
    e16, e32 = rel(out, out16), rel(out, out32)
    print(f'bf16 logits rel err vs emulated {e16:.2e}, vs fp32 {e32:.2e}; loss {loss.item():.6f} emulated '
          f'{loss16.item():.6f} fp32 {loss32.item():.6f}')
    assert e32 < 3e-2
    assert e16 < e32
    assert abs(loss.item() - loss32.item()) < 1e-2
    worst = 1.0
    for k, p in net.module.named_parameters():
        if k.endswith('conv.0.bias') or k.endswith('conv.3.bias'):
            continue
        a = p.grad.detach().double().cpu().flatten()
        b = g32[k].double().flatten()
        cs = float(torch.dot(a, b) / (a.norm() * b.norm()))
        worst = min(worst, cs)
        assert cs > 0.95, (k, cs)
    print(f'bf16 worst gradient cosine similarity {worst:.4f}')


@pytest.mark.parametrize('math', ['f32', 'x3', 'x5'])
def test_split_math_siamese_model_step_meets_the_fp32_bars(dev, math):
    """The fp32-class arithmetics at model level (TOPOLOGY [64, 128], 64x64: every level on the halo kernels)
    against the fp32 oracle: logits 1e-4 relative, loss 1e-5.  Gradients: at this size a few ReLU-kink pixels
    move the max-norm gradient error to ~2e-2 for EVERY fp32 implementation (the exact-fp32 MFMA path included,
    measured 1.8e-2; x3 3.6e-2, x5 3.5e-2), so they are compared by cosine similarity (> 0.9999 per tensor; x5,
    which drops a <= 2^-18 product in every conv including the 16-channel input layer, > 0.9998: measured
    0.99987 at worst)."""
    from multimodal_siamese_cd_amd import hip
    from multimodal_siamese_cd_amd.utils import experiment_manager as em, loss_functions, networks
    from oracle import siamese_oracle as O
    cfg = em.load_cfg('debug')
    ocfg = dict(TYPE='siameseunet', TOPOLOGY=[64, 128], IN_CHANNELS=5, OUT_CHANNELS=1, S1_BANDS=[0, 1],
                S2_BANDS=[2, 1, 0])
    shapes = O.param_shapes('siameseunet', ocfg)
    P = O.deterministic_params(shapes, 3)
    B = O.fresh_buffers(shapes)
    batch = O.synthetic_batch(ocfg, 2, 64, 4)
    out32, loss32, g32 = _oracle_step(P, B, batch, ocfg, False)
    cfg.MODEL.CONV_MATH = math
    net = networks.create_network(cfg).to(dev)
    assert net.module.conv_math == math
    with torch.no_grad():
        for k, p in net.module.named_parameters():
            p.copy_(P[k])
    net.train()
    out = net(batch['x_t1'].to(dev), batch['x_t2'].to(dev))
    loss = loss_functions.get_criterion('PowerJaccardLoss')(out, batch['y_change'].to(dev))
    loss.backward()
    e = rel(out, out32)
    cos = {}
    for k, p in net.module.named_parameters():
        if k.endswith('conv.0.bias') or k.endswith('conv.3.bias'):
            continue
        a, b = p.grad.detach().double().cpu().flatten(), g32[k].double().flatten()
        cos[k] = float(torch.dot(a, b) / (a.norm() * b.norm()))
    worst = min(cos.values())
    print(f'{math} logits rel err {e:.2e}, loss {loss.item():.7f} vs {loss32.item():.7f}, '
          f'worst gradient cosine {worst:.6f}')
    assert e < 1e-4
    assert abs(loss.item() - loss32.item()) < 1e-5
    assert worst > (0.9998 if math == 'x5' else 0.9999), sorted(cos.items(), key=lambda kv: kv[1])[:4]
