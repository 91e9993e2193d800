"""SCD_MATH_H2 (two-term fp16 split with power-of-two operand scaling, three MFMA products) on MI355X.

The arithmetic is fp32-accurate only if every operand bound really bounds its operand, so besides the kernels'
accuracy against fp64 these tests pin the bound producers (BatchNorm statistics, BatchNorm backward, absmax),
the weight split and its per-row scales, the routing (no bound -> x3), and a whole training step against the
CPU oracle with every 32-channel conv on the h2 kernels.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from _parity import branch_matched_reference, check_branch_matched
from oracle.golden import rel_err

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def dev():
    from multimodal_siamese_cd_amd import hip
    hip.load_library()
    d = torch.device('cuda:0')
    hip.ensure_device(torch.empty(1, device=d))
    return d


@pytest.fixture
def h2(dev):
    from multimodal_siamese_cd_amd import hip
    prev = hip.set_conv_math('h2')
    yield
    hip.set_conv_math(prev)


def rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


def nchw(t):
    return t.permute(0, 3, 1, 2).contiguous()


def nhwc_t(t):
    return t.permute(0, 2, 3, 1).contiguous()


def absmax(t, dev, loose=1.0):
    from multimodal_siamese_cd_amd import hip
    b = torch.zeros(1, device=dev)
    hip.absmax_bound(hip.nhwc(t), b)
    return b * loose


def test_h2_weight_split_reconstructs_rows(dev, h2):
    """h + m of each scaled row equals w * 2^k to 2^-22 relative; the inverse scales are powers of two that put the
    row max in [2^14, 2^15); zero rows get scale 1; the batched pack writes the same split as the standalone one."""
    from multimodal_siamese_cd_amd import hip
    g = torch.Generator().manual_seed(1)
    co, ci = 96, 64
    w = (torch.randn(co, ci, 3, 3, generator=g) * 10 ** (3 * torch.rand(co, 1, 1, 1, generator=g) - 1.5))
    w[5] = 0.0
    wd = w.to(dev)
    wpk = hip.pack_conv3x3(wd, 0)
    sp = wpk._x3
    K, NB = 9 * ci, (co + 31) // 32
    plane = NB * 32 * K
    hm = sp[:2 * plane].view(torch.float16).float().cpu()
    inv = sp[2 * plane:2 * plane + 2 * NB * 32].view(torch.float32).cpu()
    assert torch.all(inv[co:] == 1.0) and inv[5] == 1.0
    e = torch.log2(inv[:co])
    assert torch.equal(e, e.round())
    # fragment order -> [n][K]: e = (nb*KS + ks)*64 + lane, 8 k per slot
    KS = K // 16
    slots = torch.arange(NB * KS * 64)
    lane, fk = slots % 64, slots // 64
    nb, ks = fk // KS, fk % KS
    n = nb * 32 + lane % 32
    k0 = ks * 16 + 8 * (lane // 32)
    rec = torch.zeros(NB * 32, K)
    for p in range(2):
        vals = hm[p * plane:(p + 1) * plane].view(-1, 8)
        for j in range(8):
            rec[n, k0 + j] += vals[:, j]
    packed = wpk.view(co, K).cpu()
    scaled = packed / inv[:co, None]
    assert (scaled.abs().max(1).values[torch.arange(co) != 5] < 2 ** 15).all()
    assert (scaled.abs().max(1).values[torch.arange(co) != 5] >= 2 ** 14).all()
    err = (rec[:co] - scaled).abs() / scaled.abs().max(1, keepdim=True).values.clamp_min(1e-30)
    assert err.max().item() < 2 ** -21
    # the batched pack (one launch for all jobs) writes the same bytes
    multi = hip.pack_conv3x3_multi([(wd, 0, ci), (wd, 1, ci)])
    used = lambda t, rows, k: t[:2 * ((rows + 31) // 32 * 32) * k + 2 * ((rows + 31) // 32 * 32)]  # planes + scales
    assert torch.equal(used(multi[0]._x3, co, K), used(sp, co, K))
    assert torch.equal(used(multi[1]._x3, ci, 9 * co), used(hip.pack_conv3x3(wd, 1)._x3, ci, 9 * co))


@pytest.mark.parametrize('ci,co', [(64, 128), (256, 256), (128, 64), (512, 512)])
@pytest.mark.parametrize('loose', [1.0, 1024.0])
def test_h2_halo_accuracy_vs_fp64(dev, ci, co, loose):
    """Forward, data grad and weight grad under h2 against fp64 on data spread over 1e-2..1e2, with exact and
    1024x loose bounds: within 2x of the fp32-MFMA kernels' error (the representation error, 2^-22, sits below
    fp32 accumulation noise)."""
    from multimodal_siamese_cd_amd import hip
    g = torch.Generator().manual_seed(ci + co)
    n, h, w = 2, 32, 32
    spread = lambda *s: (torch.randn(*s, generator=g, dtype=torch.float64)
                         * 10 ** (4 * torch.rand(*s, generator=g, dtype=torch.float64) - 2)).float()
    x, dy = spread(n, h, w, ci), spread(n, h, w, co)
    wt = (torch.randn(co, ci, 3, 3, generator=g, dtype=torch.float64) / (3 * ci ** 0.5)).float()
    ref_y = nhwc_t(F.conv2d(nchw(x).double(), wt.double(), None, padding=1))
    ref_dx = nhwc_t(torch.nn.grad.conv2d_input((n, ci, h, w), wt.double(), nchw(dy).double(), padding=1))
    ref_dw = torch.nn.grad.conv2d_weight(nchw(x).double(), (co, ci, 3, 3), nchw(dy).double(), padding=1)
    errs = {}
    for m in ('f32', 'h2'):
        prev = hip.set_conv_math(m)
        try:
            xd, dyd, wd = x.to(dev), dy.to(dev), wt.to(dev)
            xb, db = (absmax(xd, dev, loose), absmax(dyd, dev, loose)) if m == 'h2' else (None, None)
            y = torch.empty(n, h, w, co, device=dev)
            src = hip.nhwc(xd)
            wpk = hip.pack_conv3x3(wd, 0)
            if m == 'h2':
                assert hip.igemm_arith(src, h, w, 1, hip.TAPS_3X3, wpk, co, hip.nhwc(y), src_bound=xb) == 'h2'
            hip.conv_igemm(src, h, w, 1, hip.TAPS_3X3, wpk, co, None, hip.nhwc(y), src_bound=xb)
            dx = torch.empty(n, h, w, ci, device=dev)
            hip.conv_igemm(hip.nhwc(dyd), h, w, 1, hip.TAPS_3X3, hip.pack_conv3x3(wd, 1), ci, None, hip.nhwc(dx),
                           src_bound=db)
            d, nsplit, nbytes = hip.wgrad_plan(hip.nhwc(dyd), hip.nhwc(xd), 1, hip.TAPS_3X3, None, db, xb)
            if m == 'h2':
                assert hip.wgrad_arith(d) == 'h2'
            slabs = torch.empty(nbytes // 4, device=dev)
            hip.conv_wgrad(d, slabs)
            dw = torch.empty(co, ci, 3, 3, device=dev)
            hip.wgrad_finalize(slabs, nsplit, co, 9, ci, 0, ci, dw)
        finally:
            hip.set_conv_math(prev)
        errs[m] = (rel(y, ref_y), rel(dx, ref_dx), rel(dw, ref_dw))
    print(errs)
    for k in range(3):
        assert errs['h2'][k] <= 2 * errs['f32'][k] + 1e-7, (k, errs)


@pytest.mark.parametrize('math', ['h2', 'bf16'])
@pytest.mark.parametrize('n,h,w,ci,co', [(2, 8, 32, 64, 128), (1, 6, 48, 128, 384), (3, 4, 16, 64, 256)])
def test_wgrad_128_row_blocks(dev, monkeypatch, math, n, h, w, ci, co):
    """The 128-row weight-grad blocks (two wave groups sharing one staged X halo; SCD_TUNE_WGRAD_R64 keeps 64-row blocks)
    against fp64, with split-K slabs and a row count that is an odd multiple of 128: h2 within 2x of the 64-row
    kernel's error (and fp32-level), bf16 at bf16 accuracy; bit-identical to the 64-row blocks at equal split-K."""
    from multimodal_siamese_cd_amd import hip
    g = torch.Generator().manual_seed(n * co + ci)
    x = torch.randn(n, h, w, ci, generator=g)
    dy = torch.randn(n, h, w, co, generator=g) * 10 ** (2 * torch.rand(n, h, w, co, generator=g) - 1)
    ref = torch.nn.grad.conv2d_weight(nchw(x).double(), (co, ci, 3, 3), nchw(dy).double(), padding=1)
    prev = hip.set_conv_math(math)
    try:
        xd, dyd = x.to(dev), dy.to(dev)
        xb, db = (absmax(xd, dev), absmax(dyd, dev)) if math == 'h2' else (None, None)
        out, dws = {}, {}
        for r128 in ('0', '1'):
            with hip.conv_scope(tune=0 if r128 == '1' else hip.TUNE_WGRAD_R64):
                d, nsplit, nbytes = hip.wgrad_plan(hip.nhwc(dyd), hip.nhwc(xd), 1, hip.TAPS_3X3, None, db, xb)
            assert hip.wgrad_arith(d) == math
            assert hip.wgrad_rows_per_block(d) == (128 if r128 == '1' else 64)
            slabs = torch.full((nbytes // 4,), float('nan'), device=dev)
            hip.conv_wgrad(d, slabs)
            dw = torch.empty(co, ci, 3, 3, device=dev)
            hip.wgrad_finalize(slabs, nsplit, co, 9, ci, 0, ci, dw)
            out[r128] = rel(dw, ref)
            dws[r128] = (nsplit, dw)
    finally:
        hip.set_conv_math(prev)
    print(out)
    if dws['0'][0] == dws['1'][0]:  # same split-K: every element sums the same products in the same order
        assert torch.equal(dws['0'][1], dws['1'][1])
    if math == 'h2':
        assert out['1'] <= 2 * out['0'] + 1e-7 and out['1'] < 1e-5, out
    else:
        assert out['1'] < 2e-2 and out['0'] < 2e-2, out


def test_h2_without_bound_runs_x3(dev, h2):
    """No bound: the conv reports and runs x3 (fp32 weights split on the fly), the result stays fp32-accurate."""
    from multimodal_siamese_cd_amd import hip
    g = torch.Generator().manual_seed(5)
    n, h, w, ci, co = 2, 16, 16, 64, 64
    x = torch.randn(n, h, w, ci, generator=g)
    wt = torch.randn(co, ci, 3, 3, generator=g) / 24
    ref = nhwc_t(F.conv2d(nchw(x), wt, None, padding=1))
    xd = x.to(dev)
    y = torch.empty(n, h, w, co, device=dev)
    wpk = hip.pack_conv3x3(wt.to(dev), 0)
    assert hip.igemm_arith(hip.nhwc(xd), h, w, 1, hip.TAPS_3X3, wpk, co, hip.nhwc(y)) == 'x3'
    hip.conv_igemm(hip.nhwc(xd), h, w, 1, hip.TAPS_3X3, wpk, co, None, hip.nhwc(y))
    assert rel(y, ref) < 1e-5
    d, _, _ = hip.wgrad_plan(hip.nhwc(y), hip.nhwc(xd), 1, hip.TAPS_3X3)
    assert hip.wgrad_arith(d) == 'x3'


def test_h2_underestimated_bound_is_detectable(dev, h2):
    """The contract's failure mode: a bound far below the data overflows fp16 -> non-finite outputs (never a
    silently wrong finite answer of fp32 size)."""
    from multimodal_siamese_cd_amd import hip
    n, h, w, ci, co = 1, 16, 16, 32, 64
    xd = torch.full((n, h, w, ci), 1000.0, device=dev)
    wt = torch.full((co, ci, 3, 3), 0.01, device=dev)
    y = torch.empty(n, h, w, co, device=dev)
    bad = torch.full((1,), 1e-3, device=dev)
    hip.conv_igemm(hip.nhwc(xd), h, w, 1, hip.TAPS_3X3, hip.pack_conv3x3(wt, 0), co, None, hip.nhwc(y), src_bound=bad)
    assert not torch.isfinite(y).all()


@pytest.mark.parametrize('n,h,w,c,nseg', [(4, 16, 16, 64, 2), (2, 33, 17, 32, 1), (6, 8, 8, 512, 2)])
def test_bound_producers(dev, n, h, w, c, nseg):
    """BatchNorm statistics bound their ReLU output (and are not looser than sqrt(n) x the data's range);
    the BatchNorm backward raises its bound to exactly max |dy|; absmax (plain and through BN + ReLU) is exact."""
    from multimodal_siamese_cd_amd import hip
    g = torch.Generator().manual_seed(n * c + h)
    y = (torch.randn(n, h, w, c, generator=g) * 3 + 1).to(dev)
    y[0, 0, 0, 0] = 40.0  # an outlier
    gamma = (torch.rand(c, generator=g) + 0.5).to(dev)
    beta = torch.randn(c, generator=g).to(dev)
    smean, sinv, scale, shift = (torch.empty(nseg * c, device=dev) for _ in range(4))
    ws = torch.empty(hip.bn_workspace_bytes(n, h, w, c, nseg), dtype=torch.uint8, device=dev)
    ab = torch.zeros(1, device=dev)
    hip.bn_train_stats(hip.nhwc(y), nseg, gamma, beta, 1e-5, 0.1, False, None, None, smean, sinv, scale, shift, ws,
                       act_bound=ab)
    seg = n // nseg
    act = torch.cat([torch.relu(y[s * seg:(s + 1) * seg] * scale[s * c:(s + 1) * c] + shift[s * c:(s + 1) * c])
                     for s in range(nseg)])
    amax = act.abs().max().item()
    assert ab.item() >= amax
    assert ab.item() <= 1.01 * (gamma.abs().max().item() * (n * h * w / nseg) ** 0.5 + beta.abs().max().item())
    ex = torch.zeros(1, device=dev)
    hip.absmax_bound(hip.nhwc(y), ex, nseg, scale, shift)
    assert ex.item() == amax
    ex.zero_()
    hip.absmax_bound(hip.nhwc(y), ex)
    assert ex.item() == y.abs().max().item()
    # backward: dy_bound == max |dy|
    da = torch.randn(n, h, w, c, generator=g).to(dev)
    dyo = torch.empty_like(y)
    dg, dbt = torch.empty(c, device=dev), torch.empty(c, device=dev)
    db = torch.zeros(1, device=dev)
    hip.bn_relu_backward(hip.nhwc(y), hip.nhwc(da), nseg, smean, sinv, gamma, scale, shift, dg, dbt, None,
                         hip.nhwc(dyo), ws, dy_bound=db)
    assert db.item() == dyo.abs().max().item()


def _record_arith(monkeypatch, dev):
    """Wrap hip.conv_igemm / hip.conv_wgrad to record, per launch, its arithmetic and the one it would have with
    bounds on every operand (h2 where the library's h2 kernels take the shape)."""
    from multimodal_siamese_cd_amd import hip
    seen = []
    orig_igemm, orig_wgrad = hip.conv_igemm, hip.conv_wgrad
    one = torch.ones(1, device=dev)

    def igemm(src, out_h, out_w, stride, taps, wpk, n_out, bias, dst, store_mode=0, **kw):
        a = hip.igemm_arith(src, out_h, out_w, stride, taps, wpk, n_out, dst, store_mode, src_bound=kw.get('src_bound'))
        b = hip.igemm_arith(src, out_h, out_w, stride, taps, wpk, n_out, dst, store_mode, src_bound=one)
        seen.append(('igemm', src.c, n_out, out_h, out_w, a, b))
        return orig_igemm(src, out_h, out_w, stride, taps, wpk, n_out, bias, dst, store_mode, **kw)

    def wgrad(d, slabs):
        e = hip.WGRAD.from_buffer_copy(d)
        e.rows_bound = e.src_bound = one.data_ptr()
        seen.append(('wgrad', d.src.c, d.rows.c, d.rows.h, d.rows.w, hip.wgrad_arith(d), hip.wgrad_arith(e)))
        return orig_wgrad(d, slabs)

    monkeypatch.setattr(hip, 'conv_igemm', igemm)
    monkeypatch.setattr(hip, 'conv_wgrad', wgrad)
    return seen


@pytest.mark.parametrize('model,topo,size', [('siameseunet', [32, 64, 128], 64), ('siameseunet', [64, 128], 96),
                                             ('dualstreamunet', [32, 64], 64), ('unet', [32, 64], 48),
                                             ('siameseunet', [64, 128, 256, 512], 256)])
def test_h2_model_step_matches_oracle(dev, monkeypatch, model, topo, size):
    """A training step with every conv the h2 kernels take on h2 (checked launch by launch, none left without a
    bound): logits within 1e-4 and loss within 1e-5 of the fp32 CPU oracle, BatchNorm running statistics within
    1e-5.  Gradients of the h2 run (and of the x3 run beside it) within 1e-3 of the fp64 oracle following that run's
    own ReLU / MaxPool branches (tests/_parity.py), every tensor, at every size including the full model."""
    from multimodal_siamese_cd_amd import engine
    from multimodal_siamese_cd_amd.utils import experiment_manager, loss_functions, networks
    from oracle import siamese_oracle as O
    ocfg = dict(TOPOLOGY=topo, IN_CHANNELS=5, OUT_CHANNELS=1, S1_BANDS=[0, 1], S2_BANDS=[2, 1, 0])
    shapes = O.param_shapes(model, ocfg)
    P = O.deterministic_params(shapes, 7)
    b = O.synthetic_batch(ocfg, 2, size, 8)
    cfg = experiment_manager.new_config()
    cfg.MODEL.TYPE, cfg.MODEL.IN_CHANNELS, cfg.MODEL.OUT_CHANNELS = model, 5, 1
    cfg.MODEL.TOPOLOGY = topo
    cfg.DATALOADER.S1_BANDS, cfg.DATALOADER.S2_BANDS = [0, 1], [2, 1, 0]
    crit = loss_functions.get_criterion('PowerJaccardLoss')
    runs = {}
    for m in ('x3', 'h2'):
        cfg.MODEL.CONV_MATH = m if m == 'x3' else None  # None: MODEL.PRECISION fp32 -> h2 (create_network)
        net = networks.create_network(cfg)
        assert net.module.conv_math == m
        with torch.no_grad():
            for k, p in net.module.named_parameters():
                p.copy_(P[k])
        net.to(dev).train()
        seen = _record_arith(monkeypatch, dev)
        with engine.trace_bn() as trace:
            out = net(b['x_t1'].to(dev), b['x_t2'].to(dev))
        loss = crit(out, b['y_change'].to(dev))
        loss.backward()
        monkeypatch.undo()
        if m == 'h2':
            h2_shapes = [s for s in seen if s[6] == 'h2']
            print(f'{len(h2_shapes)} of {len(seen)} conv launches take the h2 kernels')
            assert h2_shapes and all(s[5] == 'h2' for s in h2_shapes), [s for s in h2_shapes if s[5] != 'h2']
        runs[m] = (out.detach().cpu().numpy(), loss.item(),
                   {k: p.grad.cpu().double() for k, p in net.module.named_parameters()},
                   {k: v.cpu() for k, v in net.module.state_dict().items()}, trace, net.module)
    B32 = O.fresh_buffers(shapes)
    with torch.no_grad():
        r = O.forward(model, P, B32, b['x_t1'], b['x_t2'], ocfg, True)
    lr = O.power_jaccard_loss(r, b['y_change']).item()
    r = r.numpy()
    o, l, g, sd = runs['h2'][:4]
    print(f"logits rel err vs the fp32 oracle: h2 {rel_err(o, r):.2e}, x3 {rel_err(runs['x3'][0], r):.2e}")
    assert rel_err(o, r) < 1e-4
    assert abs(l - lr) < 1e-5
    order = [k for k, _ in net.module.named_parameters()]
    for m in ('x3', 'h2'):
        _, _, ref = branch_matched_reference(model, P, b, ocfg, runs[m][4], runs[m][5],
                                             lambda out, bt: O.power_jaccard_loss(out, bt['y_change']))
        bad = check_branch_matched(runs[m][2], ref, order, 1e-3)
        assert not bad, (m, bad)
    for k, v in B32.items():
        if k.endswith('running_mean') or k.endswith('running_var'):
            assert rel_err(sd[k].numpy(), v.numpy()) < 1e-5, k


def test_h2_eval_forward_matches_oracle(dev, h2):
    """Eval mode (running statistics): the bounds come from absmax passes; logits within 1e-4 of the oracle."""
    from multimodal_siamese_cd_amd.utils import experiment_manager, networks
    from oracle import siamese_oracle as O
    topo = [32, 64]
    ocfg = dict(TOPOLOGY=topo, IN_CHANNELS=5, OUT_CHANNELS=1, S1_BANDS=[0, 1], S2_BANDS=[2, 1, 0])
    shapes = O.param_shapes('siameseunet', ocfg)
    P = O.deterministic_params(shapes, 3)
    B = O.fresh_buffers(shapes)
    g = torch.Generator().manual_seed(0)
    for k in B:
        if k.endswith('running_mean'):
            B[k] = torch.randn(B[k].shape, generator=g) * 0.1
        elif k.endswith('running_var'):
            B[k] = torch.rand(B[k].shape, generator=g) + 0.5
    b = O.synthetic_batch(ocfg, 2, 64, 4)
    cfg = experiment_manager.new_config()
    cfg.MODEL.TYPE, cfg.MODEL.IN_CHANNELS, cfg.MODEL.OUT_CHANNELS = 'siameseunet', 5, 1
    cfg.MODEL.TOPOLOGY = topo
    cfg.DATALOADER.S1_BANDS, cfg.DATALOADER.S2_BANDS = [0, 1], [2, 1, 0]
    net = networks.create_network(cfg)
    sd = net.module.state_dict()
    with torch.no_grad():
        for k, v in {**P, **B}.items():
            sd[k].copy_(v)
    net.to(dev).eval()
    with torch.no_grad():
        out = net(b['x_t1'].to(dev), b['x_t2'].to(dev))
        ref = O.forward('siameseunet', P, B, b['x_t1'], b['x_t2'], ocfg, False)
    assert rel_err(out.cpu().numpy(), ref.numpy()) < 1e-4


@pytest.mark.parametrize('tiny_exp', [-12, -18, -24, -30])
def test_h2_wide_dynamic_range(dev, h2, tiny_exp):
    """Operands whose bulk sits far below their max (one outlier at 1.0, the rest ~2^tiny_exp): the scaled terms of
    the bulk fall towards or below the fp16 normal range.  Forward, data grad (the outlier in dY) and weight grad
    (the outlier in dY) must stay fp32-accurate on the outputs the outlier does not reach: the low term of activation
    and gradient operands is pre-scaled by 2^11, which keeps 22 bits down to 2^-28 of the bound."""
    from multimodal_siamese_cd_amd import hip
    g = torch.Generator().manual_seed(-tiny_exp)
    n, h, w, ci, co = 1, 16, 32, 64, 64
    wide = lambda c: (lambda t: (t.__setitem__((0, 0, 0, 0), 1.0), t)[1])(
        (torch.rand(n, h, w, c, generator=g, dtype=torch.float64) + 0.5) * 2.0 ** tiny_exp).float()
    x, dy = wide(ci), wide(co)
    xn = torch.rand(n, h, w, ci, generator=g) + 0.5
    wt = torch.randn(co, ci, 3, 3, generator=g) / 17
    ref_y = nhwc_t(F.conv2d(nchw(x).double(), wt.double(), None, padding=1))
    ref_dx = nhwc_t(torch.nn.grad.conv2d_input((n, ci, h, w), wt.double(), nchw(dy).double(), padding=1))
    xd, dyd, xnd, wd = x.to(dev), dy.to(dev), xn.to(dev), wt.to(dev)
    y = torch.empty(n, h, w, co, device=dev)
    hip.conv_igemm(hip.nhwc(xd), h, w, 1, hip.TAPS_3X3, hip.pack_conv3x3(wd, 0), co, None, hip.nhwc(y),
                   src_bound=absmax(xd, dev))
    dx = torch.empty(n, h, w, ci, device=dev)
    hip.conv_igemm(hip.nhwc(dyd), h, w, 1, hip.TAPS_3X3, hip.pack_conv3x3(wd, 1), ci, None, hip.nhwc(dx),
                   src_bound=absmax(dyd, dev))
    far = lambda a, r: ((a.cpu().double()[:, 4:, 4:] - r[:, 4:, 4:]).abs().max() / r[:, 4:, 4:].abs().max()).item()
    # weight grad: the outlier pixel's row of dY excluded by zeroing its neighbourhood in x (no contribution)
    xn2 = xnd.clone()
    xn2[:, :3, :3] = 0
    ref_dw = torch.nn.grad.conv2d_weight(nchw(xn2.cpu()).double(), (co, ci, 3, 3), nchw(dy).double(), padding=1)
    d, nsplit, nbytes = hip.wgrad_plan(hip.nhwc(dyd), hip.nhwc(xn2), 1, hip.TAPS_3X3, None, absmax(dyd, dev),
                                       absmax(xn2, dev))
    assert hip.wgrad_arith(d) == 'h2'
    slabs = torch.empty(nbytes // 4, device=dev)
    hip.conv_wgrad(d, slabs)
    dw = torch.empty(co, ci, 3, 3, device=dev)
    hip.wgrad_finalize(slabs, nsplit, co, 9, ci, 0, ci, dw)
    errs = (far(y, ref_y), far(dx, ref_dx), rel(dw, ref_dw))
    print(f'bulk at 2^{tiny_exp}: rel err fwd {errs[0]:.2e} dgrad {errs[1]:.2e} wgrad {errs[2]:.2e}')
    assert max(errs) < 1e-5, errs


@pytest.mark.parametrize('n,h,w,ci,co', [(2, 8, 8, 64, 64), (3, 5, 7, 128, 64)])
def test_convT_dst_bound(dev, h2, n, h, w, ci, co):
    """The ConvTranspose forward raises dst_bound to exactly max |output| while it stores into the concat slice (the
    bound of the decoder's concat without a pass over it); other store modes refuse the request."""
    from multimodal_siamese_cd_amd import hip
    g = torch.Generator().manual_seed(n * h + w)
    x = torch.randn(n, h, w, ci, generator=g).to(dev)
    wt = (torch.randn(ci, co, 2, 2, generator=g) / 8).to(dev)
    b = torch.randn(co, generator=g).to(dev)
    cat = torch.zeros(n, 2 * h, 2 * w, co + 32, device=dev)
    bound = torch.full((1,), 0.5, device=dev)  # an earlier (smaller) bound is raised, never lowered
    hip.conv_igemm(hip.nhwc(x), h, w, 1, hip.TAPS_1, hip.pack_convT2x2(wt, 0), 4 * co, b, hip.nhwc(cat, 32, co),
                   store_mode=1, dst_bound=bound)
    up = cat[..., 32:]
    ref = F.conv_transpose2d(nchw(x).cpu(), wt.cpu(), b.cpu(), stride=2)
    assert rel(nchw(up), ref) < 1e-5
    assert bound.item() == max(0.5, up.abs().max().item())
    y = torch.empty(n, h, w, co, device=dev)
    with pytest.raises(RuntimeError, match='dst_bound'):
        hip.conv_igemm(hip.nhwc(y), h, w, 1, hip.TAPS_3X3, hip.pack_conv3x3(torch.randn(co, co, 3, 3, device=dev), 0),
                       co, None, hip.nhwc(torch.empty_like(y)), dst_bound=bound)


@pytest.mark.parametrize('n,h,w,ci,co', [(2, 8, 8, 64, 64), (3, 5, 7, 128, 64), (8, 64, 64, 64, 64),
                                         (2, 16, 16, 256, 128), (1, 4, 4, 512, 512)])
def test_convT_gather16(dev, h2, n, h, w, ci, co):
    """The ConvTranspose forward (1 tap, pixel-shuffle store) and data grad (4 taps, stride-2 gather) with a source
    bound take the h2 gather16 kernel: fp32-accurate against fp64 (tiles 128x128 / 128x64 / 64x128, ragged pixel
    counts), dst_bound raised to exactly max |up|; without a bound they stay on x3 and agree."""
    from multimodal_siamese_cd_amd import hip
    g = torch.Generator().manual_seed(n * h * w + ci)
    x = torch.randn(n, h, w, ci, generator=g).to(dev)
    wt = (torch.randn(ci, co, 2, 2, generator=g) / 8).to(dev)
    b = torch.randn(co, generator=g).to(dev)
    wf, wb = hip.pack_convT2x2(wt, 0), hip.pack_convT2x2(wt, 1)
    cat = torch.zeros(n, 2 * h, 2 * w, co + 32, device=dev)
    xb = absmax(x, dev, 3.0)  # a loose bound is as good (only the absolute floor moves)
    assert hip.igemm_arith(hip.nhwc(x), h, w, 1, hip.TAPS_1, wf, 4 * co, hip.nhwc(cat, 32, co), store_mode=1,
                           src_bound=xb) == 'h2'
    bound = torch.zeros(1, device=dev)
    hip.conv_igemm(hip.nhwc(x), h, w, 1, hip.TAPS_1, wf, 4 * co, b, hip.nhwc(cat, 32, co), store_mode=1,
                   src_bound=xb, dst_bound=bound)
    up = cat[..., 32:]
    ref = F.conv_transpose2d(nchw(x).cpu().double(), wt.cpu().double(), b.cpu().double(), stride=2)
    assert rel(nchw(up), ref) < 2e-6
    assert torch.equal(cat[..., :32], torch.zeros_like(cat[..., :32]))
    assert bound.item() == up.abs().max().item()
    # data grad: g_up read from a channel slice of a wider buffer (the decoder's g_cat)
    gcat = torch.randn(n, 2 * h, 2 * w, co + 32, generator=g).to(dev)
    gub = absmax(gcat, dev)
    assert hip.igemm_arith(hip.nhwc(gcat, 32, co), h, w, 2, hip.TAPS_2X2, wb, ci, hip.nhwc(x), src_bound=gub) == 'h2'
    gx = torch.empty(n, h, w, ci, device=dev)
    hip.conv_igemm(hip.nhwc(gcat, 32, co), h, w, 2, hip.TAPS_2X2, wb, ci, None, hip.nhwc(gx), src_bound=gub)
    xr = nchw(x).cpu().double().requires_grad_()
    wr = wt.cpu().double().requires_grad_()
    F.conv_transpose2d(xr, wr, None, stride=2).backward(nchw(gcat[..., 32:]).cpu().double())
    assert rel(nchw(gx), xr.grad) < 2e-6
    gx3 = torch.empty_like(gx)  # no bound: the x3 kernel, same values to fp32 rounding
    hip.conv_igemm(hip.nhwc(gcat, 32, co), h, w, 2, hip.TAPS_2X2, wb, ci, None, hip.nhwc(gx3))
    assert rel(gx3, gx) < 2e-6
    # weight grad: rows = the ConvT input, src = g_up gathered with stride 2, both bounded -> generic h2 weight grad
    for bounds, arith in (((xb, gub), 'h2'), ((None, None), 'x3')):
        d, nsplit, nbytes = hip.wgrad_plan(hip.nhwc(x), hip.nhwc(gcat, 32, co), 2, hip.TAPS_2X2, None, *bounds)
        assert hip.wgrad_arith(d) == arith
        slabs = torch.empty(nbytes // 4, device=dev)
        hip.conv_wgrad(d, slabs)
        gw = torch.empty(ci, co, 2, 2, device=dev)
        hip.wgrad_finalize(slabs, nsplit, ci, 4, co, 1, co, gw)
        assert rel(gw, wr.grad) < 2e-6, arith


@pytest.mark.parametrize('bounded', [False, True])
def test_convT_dst_bound_seed(dev, h2, bounded):
    """ABI 9: the ConvTranspose forward folds dst_bound_seed into dst_bound inside the launch (the decoder seeds its
    concat bound with the skip's bound without a device copy): dst_bound ends at max(seed, max |up|), the seed float is
    left as it was; on the x3 per-tap kernel (no source bound) and the h2 gather16 kernel; a seed without dst_bound is
    refused."""
    from multimodal_siamese_cd_amd import hip
    g = torch.Generator().manual_seed(17)
    n, h, w, ci, co = 2, 16, 16, 64, 64
    x = torch.randn(n, h, w, ci, generator=g).to(dev)
    wt = (torch.randn(ci, co, 2, 2, generator=g) / 8).to(dev)
    b = torch.randn(co, generator=g).to(dev)
    wf = hip.pack_convT2x2(wt, 0)
    xb = absmax(x, dev) if bounded else None
    for seed_val in (1e3, float(torch.tensor(1e-3))):  # above and below the output's max (fp32 values)
        cat = torch.zeros(n, 2 * h, 2 * w, co + 32, device=dev)
        seed = torch.full((1,), seed_val, device=dev)
        bound = torch.zeros(1, device=dev)
        assert hip.igemm_arith(hip.nhwc(x), h, w, 1, hip.TAPS_1, wf, 4 * co, hip.nhwc(cat, 32, co), store_mode=1,
                               src_bound=xb) == ('h2' if bounded else 'x3')
        hip.conv_igemm(hip.nhwc(x), h, w, 1, hip.TAPS_1, wf, 4 * co, b, hip.nhwc(cat, 32, co), store_mode=1,
                       src_bound=xb, dst_bound=bound, dst_bound_seed=seed)
        assert bound.item() == max(seed_val, cat[..., 32:].abs().max().item())
        assert seed.item() == seed_val
    with pytest.raises(RuntimeError, match='dst_bound_seed'):
        hip.conv_igemm(hip.nhwc(x), h, w, 1, hip.TAPS_1, wf, 4 * co, b, hip.nhwc(cat, 32, co), store_mode=1,
                       src_bound=xb, dst_bound_seed=seed)


def test_halo16_dst_bound(dev, h2):
    """A bounded h2 3x3 conv raises dst_bound to exactly max |stored output| (the decoder's concat-gradient data
    grad hands it to the ConvTranspose data grad); without the halo16 kernel the request is refused."""
    from multimodal_siamese_cd_amd import hip
    g = torch.Generator().manual_seed(5)
    n, h, w, ci, co = 2, 32, 32, 64, 128
    x = torch.randn(n, h, w, ci, generator=g).to(dev)
    wt = (torch.randn(co, ci, 3, 3, generator=g) / 24).to(dev)
    wpk = hip.pack_conv3x3(wt, 0)
    y = torch.empty(n, h, w, co, device=dev)
    bound = torch.zeros(1, device=dev)
    assert hip.igemm_arith(hip.nhwc(x), h, w, 1, hip.TAPS_3X3, wpk, co, hip.nhwc(y), src_bound=absmax(x, dev)) == 'h2'
    hip.conv_igemm(hip.nhwc(x), h, w, 1, hip.TAPS_3X3, wpk, co, None, hip.nhwc(y), src_bound=absmax(x, dev),
                   dst_bound=bound)
    assert bound.item() == y.abs().max().item()
    ref = F.conv2d(nchw(x).cpu().double(), wt.cpu().double(), padding=1)
    assert rel(nchw(y), ref) < 2e-6
    with pytest.raises(RuntimeError, match='dst_bound'):
        hip.conv_igemm(hip.nhwc(x), h, w, 1, hip.TAPS_3X3, wpk, co, None, hip.nhwc(y), dst_bound=bound)


@pytest.mark.parametrize('env', ['TUNE_H2_TILE64_2X2', 'TUNE_H2_TILE_2X2', 'TUNE_HALO16_WS'])
@pytest.mark.parametrize('ci,co,mode', [(64, 64, 'stats'), (32, 64, 'bn_bwd'), (64, 64, 'in_bn'), (128, 128, 'stats'),
                                        (64, 128, 'bn_bwd'), (64, 96, 'plain')])
def test_h2_tile_layouts_bit_identical(dev, h2, env, ci, co, mode):
    """The 1 x N wave layouts of the h2 halo conv (the library's choice) and the 2 x 2 layouts they replace
    accumulate every output in the same order and reduce the epilogue statistics in groups of 64 pixels in both:
    outputs, BatchNorm-statistics records and BatchNorm-backward records are bit-identical."""
    from multimodal_siamese_cd_amd import hip
    from multimodal_siamese_cd_amd.hip import TAPS_3X3, nhwc
    n, h, w, nseg = 4, 32, 32, 2
    g = torch.Generator(device=dev).manual_seed(ci + co)
    x = torch.randn(n, h, w, ci, device=dev, generator=g)
    wpk = hip.pack_conv3x3(torch.randn(co, ci, 3, 3, device=dev, generator=g) / (3 * ci ** 0.5), 0)
    sc = torch.rand(nseg * ci, device=dev, generator=g) + 0.5
    sh = torch.randn(nseg * ci, device=dev, generator=g) * 0.1
    bound = x.abs().max().reshape(1) * (2.0 if mode == 'in_bn' else 1.0)
    yb = torch.randn(n, h, w, co, device=dev, generator=g)
    mu, iv = torch.randn(nseg * co, device=dev, generator=g) * 0.1, torch.rand(nseg * co, device=dev, generator=g) + .5
    bsc, bsh = torch.rand(nseg * co, device=dev, generator=g) + 0.5, torch.randn(nseg * co, device=dev, generator=g)
    outs = []
    # both layouts on 128-pixel tiles (64-channel sources otherwise take the 256 x 64 tile: test_h2_tile64_256_...)
    for tune in (hip.TUNE_H2_TILE64_128, hip.TUNE_H2_TILE64_128 | getattr(hip, env)):
        with hip.conv_scope(tune=tune):
            y = torch.full((n, h, w, co), 7.0, device=dev)
            extra, rec = {}, None
            if mode == 'in_bn':
                extra['in_bn'] = (sc, sh, nseg)
            elif mode == 'stats':
                nt, _ = hip.igemm_stat_tiles(nhwc(x), h, w, 1, TAPS_3X3, wpk, co, nhwc(y), src_bound=bound)
                rec = extra['stat_rec'] = torch.full((nt * co * 2,), 9.0, device=dev)
            elif mode == 'bn_bwd':
                nt, _ = hip.igemm_bn_bwd_tiles(nhwc(x), h, w, 1, TAPS_3X3, wpk, co, nhwc(y), bound)
                rec = torch.full((co * nt * 2,), 9.0, device=dev)
                extra['bn_bwd'] = (yb, nseg, mu, iv, bsc, bsh, rec)
            assert hip.igemm_arith(nhwc(x), h, w, 1, TAPS_3X3, wpk, co, nhwc(y), src_bound=bound) == 'h2'
            hip.conv_igemm(nhwc(x), h, w, 1, TAPS_3X3, wpk, co, None, nhwc(y), src_bound=bound, **extra)
            outs.append((y.cpu(), None if rec is None else rec.cpu()))
    assert torch.equal(outs[0][0], outs[1][0])
    if outs[0][1] is not None:
        assert torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize('ci,mode', [(64, 'stats'), (64, 'bn_bwd'), (64, 'in_bn'), (64, 'plain')])
def test_h2_tile64_256_matches_128(dev, h2, ci, mode):
    """The 256 x 64 tile of the 64-channel outputs of 64-channel sources (the default; 2 x 2 waves of 128 px x 32 ch on a
    16 x 16 patch) accumulates every output in the order of the 128 x 64 tile (SCD_TUNE_H2_TILE64_128): outputs are
    bit-identical; its epilogue records cover 256-pixel tiles, so their per-channel totals agree with the 128-pixel
    tiles' to fp32 summation order."""
    from multimodal_siamese_cd_amd import hip
    from multimodal_siamese_cd_amd.hip import TAPS_3X3, nhwc
    n, h, w, nseg, co = 4, 32, 32, 2, 64
    g = torch.Generator(device=dev).manual_seed(ci + 5)
    x = torch.randn(n, h, w, ci, device=dev, generator=g)
    wpk = hip.pack_conv3x3(torch.randn(co, ci, 3, 3, device=dev, generator=g) / (3 * ci ** 0.5), 0)
    sc = torch.rand(nseg * ci, device=dev, generator=g) + 0.5
    sh = torch.randn(nseg * ci, device=dev, generator=g) * 0.1
    bound = x.abs().max().reshape(1) * (2.0 if mode == 'in_bn' else 1.0)
    yb = torch.randn(n, h, w, co, device=dev, generator=g)
    mu, iv = torch.randn(nseg * co, device=dev, generator=g) * 0.1, torch.rand(nseg * co, device=dev, generator=g) + .5
    bsc, bsh = torch.rand(nseg * co, device=dev, generator=g) + 0.5, torch.randn(nseg * co, device=dev, generator=g)
    outs = []
    for tune in (hip.TUNE_H2_TILE64_128, 0):
        with hip.conv_scope(tune=tune):
            y = torch.full((n, h, w, co), 7.0, device=dev)
            extra, tot = {}, None
            if mode == 'in_bn':
                extra['in_bn'] = (sc, sh, nseg)
            elif mode == 'stats':
                nt, tp = hip.igemm_stat_tiles(nhwc(x), h, w, 1, TAPS_3X3, wpk, co, nhwc(y), src_bound=bound)
                assert tp == (128 if tune else 256)
                rec = extra['stat_rec'] = torch.full((nt * co * 2,), 9.0, device=dev)
            elif mode == 'bn_bwd':
                nt, tp = hip.igemm_bn_bwd_tiles(nhwc(x), h, w, 1, TAPS_3X3, wpk, co, nhwc(y), bound)
                assert tp == (128 if tune else 256)
                rec = torch.full((co * nt * 2,), 9.0, device=dev)
                extra['bn_bwd'] = (yb, nseg, mu, iv, bsc, bsh, rec)
            assert hip.igemm_arith(nhwc(x), h, w, 1, TAPS_3X3, wpk, co, nhwc(y), src_bound=bound) == 'h2'
            hip.conv_igemm(nhwc(x), h, w, 1, TAPS_3X3, wpk, co, None, nhwc(y), src_bound=bound, **extra)
            if mode == 'stats':  # per-channel sum of the tile means times the tile pixels = the channel total
                tot = rec.view(nt, co, 2)[..., 0].double().sum(0) * tp
            elif mode == 'bn_bwd':
                tot = rec.view(co, nt, 2).double().sum(1)
            outs.append((y.cpu(), None if tot is None else tot.cpu()))
    assert torch.equal(outs[0][0], outs[1][0])
    if outs[0][1] is not None:
        a, b = outs[0][1], outs[1][1]
        assert ((a - b).abs().max() / b.abs().max()).item() < 1e-5


@pytest.mark.parametrize('ci,co,mode', [(64, 64, 'stats'), (64, 64, 'in_bn'), (128, 64, 'bn_bwd'), (256, 64, 'in_bn'),
                                        (128, 128, 'stats'), (64, 256, 'in_bn'), (256, 128, 'bn_bwd'), (64, 96, 'plain')])
def test_halo16_weight_ring_bit_identical(dev, h2, ci, co, mode):
    """SCD_TUNE_HALO16_WRING: the h2 1 x N tiles with their weight fragments copied through a 3-slot LDS ring by LDS-DMA
    (igemm_halo16_x3's WL; counted vmcnt waits, one barrier per k-step) run the same products in the same order as the
    register path: outputs and epilogue records bit-identical, on the 256 x 64, 128 x 64 and 128 x 128 tiles, one to eight
    32-channel chunks (96 outputs: not a multiple of the tile, the register path runs)."""
    from multimodal_siamese_cd_amd import hip
    from multimodal_siamese_cd_amd.hip import TAPS_3X3, nhwc
    n, h, w, nseg = 4, 32, 48, 2
    g = torch.Generator(device=dev).manual_seed(ci * 3 + co)
    x = torch.randn(n, h, w, ci, device=dev, generator=g)
    wpk = hip.pack_conv3x3(torch.randn(co, ci, 3, 3, device=dev, generator=g) / (3 * ci ** 0.5), 0)
    sc = torch.rand(nseg * ci, device=dev, generator=g) + 0.5
    sh = torch.randn(nseg * ci, device=dev, generator=g) * 0.1
    bound = x.abs().max().reshape(1) * (2.0 if mode == 'in_bn' else 1.0)
    yb = torch.randn(n, h, w, co, device=dev, generator=g)
    mu, iv = torch.randn(nseg * co, device=dev, generator=g) * 0.1, torch.rand(nseg * co, device=dev, generator=g) + .5
    bsc, bsh = torch.rand(nseg * co, device=dev, generator=g) + 0.5, torch.randn(nseg * co, device=dev, generator=g)
    outs = []
    for tune in (0, hip.TUNE_HALO16_WRING):
        with hip.conv_scope(tune=tune):
            y = torch.full((n, h, w, co), 7.0, device=dev)
            extra, rec = {}, None
            if mode == 'in_bn':
                extra['in_bn'] = (sc, sh, nseg)
            elif mode == 'stats':
                nt, _ = hip.igemm_stat_tiles(nhwc(x), h, w, 1, TAPS_3X3, wpk, co, nhwc(y), src_bound=bound)
                rec = extra['stat_rec'] = torch.full((nt * co * 2,), 9.0, device=dev)
            elif mode == 'bn_bwd':
                nt, _ = hip.igemm_bn_bwd_tiles(nhwc(x), h, w, 1, TAPS_3X3, wpk, co, nhwc(y), bound)
                rec = torch.full((co * nt * 2,), 9.0, device=dev)
                extra['bn_bwd'] = (yb, nseg, mu, iv, bsc, bsh, rec)
            assert hip.igemm_arith(nhwc(x), h, w, 1, TAPS_3X3, wpk, co, nhwc(y), src_bound=bound) == 'h2'
            hip.conv_igemm(nhwc(x), h, w, 1, TAPS_3X3, wpk, co, None, nhwc(y), src_bound=bound, **extra)
            outs.append((y.cpu(), None if rec is None else rec.cpu()))
    assert torch.equal(outs[0][0], outs[1][0])
    if outs[0][1] is not None:
        assert torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize('variant,base', [('TUNE_HALO16_WS', 'TUNE_H2_TILE64_128'), ('TUNE_HALO16_WRING', None)])
def test_halo16_variant_training_step_bit_identical(dev, h2, variant, base):
    """The warp-specialized h2 halo kernel (SCD_TUNE_HALO16_WS: a producer wave stages the halo; both runs on
    128-pixel tiles, the only ones it has) and the weight ring (SCD_TUNE_HALO16_WRING) inside a whole training step of SiameseUNet [64, 128, 256] at 64x64: logits, loss and every gradient bit-identical to the
    default kernels."""
    from multimodal_siamese_cd_amd import hip, trainers
    from multimodal_siamese_cd_amd.utils import datasets, experiment_manager as em, networks
    cfg = em.load_cfg('debug')
    cfg.MODEL.TOPOLOGY = [64, 128, 256]
    gen = torch.Generator(device=dev).manual_seed(6)
    b = datasets.synthetic_batch(cfg, 4, dev, gen, 64)
    res = []
    t0 = getattr(hip, base) if base else 0
    for tune in (t0, t0 | getattr(hip, variant)):
        torch.manual_seed(0)
        net = networks.create_network(cfg).to(dev).train()
        with hip.conv_scope(tune=tune):
            out = net(b['x_t1'], b['x_t2'])
            loss = trainers.step_loss(cfg, out, b, net)
            loss.backward()
        res.append((out.detach(), loss.detach(), [p.grad.clone() for p in net.parameters()]))
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])
    for g0, g1 in zip(res[0][2], res[1][2]):
        assert torch.equal(g0, g1)


@pytest.mark.parametrize('n,h,w,ci,co,src_bn', [(4, 32, 32, 64, 128, False), (3, 16, 48, 128, 256, True),
                                                 (2, 32, 32, 128, 64, False), (5, 8, 64, 64, 64, True),
                                                 (1, 2, 16, 64, 128, False)])
def test_wgrad_double_buffered_bit_identical(dev, h2, n, h, w, ci, co, src_bn):
    """The double-buffered h2 halo weight grad (SCD_TUNE_WGRAD16_DB: two patch buffers, one barrier per patch, the two
    wave groups of a 128-row block staggered) against the default: identical split plan, slabs written in full
    (NaN-prefilled) and bit-identical, with and without the source BatchNorm transform, on 128- and 64-row blocks,
    including a split of a single patch."""
    from multimodal_siamese_cd_amd import hip
    g = torch.Generator().manual_seed(n * co + ci + int(src_bn))
    xd = torch.randn(n, h, w, ci, generator=g).to(dev)
    dyd = (torch.randn(n, h, w, co, generator=g) * 10 ** (2 * torch.rand(n, h, w, co, generator=g) - 1)).to(dev)
    bn = None
    if src_bn:
        sc = (torch.rand(ci, generator=g) + 0.5).to(dev)
        sh = (torch.randn(ci, generator=g) * 0.1).to(dev)
        bn = (sc, sh, 1)
    xb = (xd * (2.0 if src_bn else 1.0)).abs().max().reshape(1)
    db = dyd.abs().max().reshape(1)
    res = []
    for tune in (0, hip.TUNE_WGRAD16_DB):
        with hip.conv_scope(tune=tune):
            d, nsplit, nbytes = hip.wgrad_plan(hip.nhwc(dyd), hip.nhwc(xd), 1, hip.TAPS_3X3, bn, db, xb)
            assert hip.wgrad_arith(d) == 'h2'
            slabs = torch.full((nbytes // 4,), float('nan'), device=dev)
            hip.conv_wgrad(d, slabs)
            res.append((nsplit, hip.wgrad_rows_per_block(d), slabs.cpu()))
    assert res[0][0] == res[1][0] and res[0][1] == res[1][1]
    assert bool(torch.isfinite(res[1][2]).all())
    assert torch.equal(res[0][2], res[1][2])
