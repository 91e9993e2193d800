"""bf16 activation / gradient storage (ABI 6 scd_nhwc_t.dtype, the bf16 configs) kernel by kernel (MI355X).

Every kernel of the bf16 training step is run twice on the same values: once on fp32 views, once on bf16 views of
bf16-representable data.  Storage is the only difference, and a bf16 kernel loads exactly, computes in fp32 and rounds
once when it stores, so:
  - an NHWC output of the bf16 path equals the fp32 path's output rounded to bf16, bit for bit;
  - fp32 outputs (weight-grad slabs, BatchNorm statistics, the head's logits and parameter grads) are bit-identical;
  - reductions of a stored output (the conv-fused BatchNorm statistics, BN-backward sums and conv-bias sums) are taken
    of the stored bf16 values: checked against the same reductions in double of the bf16 tensor.
The conv kernels run the bf16 arithmetic (SCD_MATH_BF16) in both storages.
"""
import pytest
import torch

from multimodal_siamese_cd_amd import engine, hip
from multimodal_siamese_cd_amd.hip import TAPS_1, TAPS_2X2, TAPS_3X3, nhwc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def dev():
    hip.load_library()
    d = torch.device('cuda:0')
    hip.ensure_device(torch.empty(1, device=d))
    return d


@pytest.fixture(autouse=True)
def _bf16_math():
    with hip.conv_scope('bf16'):
        yield


def r16(t):
    """bf16-representable fp32 values."""
    return t.to(torch.bfloat16).float()


def randn(*shape, dev, scale=1.0, seed=0):
    g = torch.Generator(device=dev).manual_seed(seed)
    return r16(torch.randn(*shape, device=dev, generator=g) * scale)


def same_rounded(out16, out32, what=''):
    """The bf16 output is the fp32 output rounded to bf16, bit for bit."""
    assert out16.dtype == torch.bfloat16
    exp = out32.to(torch.bfloat16)
    diff = (out16.view(torch.int16) != exp.view(torch.int16)).sum().item()
    assert diff == 0, f'{what}: {diff} of {out16.numel()} bf16 elements differ from round(fp32 output)'


def rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


def _conv(x, wpk, n_out, bias=None, in_bn=None, stat=False, taps=TAPS_3X3, stride=1, out_hw=None, store_mode=0,
          dst=None, bn_bwd=None):
    n, h, w, _ = x.shape
    oh, ow = out_hw or (h, w)
    if dst is None:
        dst = torch.empty((n, oh, ow, n_out) if store_mode == 0 else (n, 2 * oh, 2 * ow, n_out // 4),
                          device=x.device, dtype=x.dtype)
    rec = None
    if stat:
        nt, tp = hip.igemm_stat_tiles(nhwc(x), oh, ow, stride, taps, wpk, n_out, nhwc(dst))
        assert nt > 0
        rec = torch.empty(nt * n_out * 2, device=x.device)
    hip.conv_igemm(nhwc(x), oh, ow, stride, taps, wpk, n_out, bias, nhwc(dst), store_mode, stat_rec=rec, in_bn=in_bn,
                   bn_bwd=bn_bwd)
    return dst, rec


@pytest.mark.parametrize('cin,cout,hw', [(64, 64, 32), (128, 128, 16), (64, 128, 32), (256, 64, 16)])
def test_conv3x3_forward(dev, cin, cout, hw):
    x = randn(2, hw, hw, cin, dev=dev)
    w = torch.randn(cout, cin, 3, 3, device=dev) / (9 * cin) ** 0.5
    b = torch.randn(cout, device=dev) * 0.1
    wpk = hip.pack_conv3x3(w, 0)
    y32, _ = _conv(x, wpk, cout, b)
    y16, rec = _conv(x.to(torch.bfloat16), wpk, cout, b, stat=True)
    assert hip.igemm_arith(nhwc(x.to(torch.bfloat16)), hw, hw, 1, TAPS_3X3, wpk, cout,
                           nhwc(y16)) == 'bf16'
    same_rounded(y16, y32, 'conv3x3 fwd')
    # fused statistics of the stored values: merged, they equal the batch statistics of the bf16 output (double)
    nt, tp = hip.igemm_stat_tiles(nhwc(x.to(torch.bfloat16)), hw, hw, 1, TAPS_3X3, wpk, cout, nhwc(y16))
    smean, sinv, scale, shift = (torch.empty(cout, device=dev) for _ in range(4))
    ws = torch.empty(hip.bn_tile_stats_workspace_bytes(nt, cout, 1), device=dev, dtype=torch.uint8)
    hip.bn_stats_from_tiles(rec, nt, tp, cout, 1, None, None, 1e-5, 0.1, False, None, None, smean, sinv, scale, shift,
                            ws)
    yd = y16.double().reshape(-1, cout)
    assert rel(smean, yd.mean(0)) < 1e-5
    assert rel(sinv, 1.0 / (yd.var(0, unbiased=False) + 1e-5).sqrt()) < 1e-5


def test_conv3x3_forward_input_bn(dev):
    """The previous BatchNorm-apply + ReLU applied while staging a bf16 source (IN_BN)."""
    cin, cout, hw = 64, 64, 32
    y0 = randn(4, hw, hw, cin, dev=dev, seed=1)
    w = torch.randn(cout, cin, 3, 3, device=dev) / (9 * cin) ** 0.5
    wpk = hip.pack_conv3x3(w, 0)
    sc = torch.rand(2 * cin, device=dev) + 0.5
    sh = torch.randn(2 * cin, device=dev) * 0.3
    assert hip.igemm_input_bn_supported(nhwc(y0.to(torch.bfloat16)), hw, hw, 1, TAPS_3X3, wpk, cout,
                                        nhwc(torch.empty(4, hw, hw, cout, device=dev, dtype=torch.bfloat16)),
                                        (sc, sh, 2))
    y32, _ = _conv(y0, wpk, cout, in_bn=(sc, sh, 2))
    y16, _ = _conv(y0.to(torch.bfloat16), wpk, cout, in_bn=(sc, sh, 2))
    same_rounded(y16, y32, 'conv3x3 fwd with input BN')


def test_conv3x3_data_grad_with_bn_backward_sums(dev):
    """A data grad whose epilogue also forms the BatchNorm-backward partial sums of its (stored) output over y."""
    c, cn, hw = 64, 128, 32
    dy = randn(2, hw, hw, cn, dev=dev, seed=2)
    w = torch.randn(cn, c, 3, 3, device=dev) / (9 * cn) ** 0.5
    wd = hip.pack_conv3x3(w, 1)
    y = randn(2, hw, hw, c, dev=dev, seed=3)
    mu, iv = torch.randn(c, device=dev) * 0.1, torch.rand(c, device=dev) + 0.5
    sc, sh = torch.rand(c, device=dev) + 0.5, torch.randn(c, device=dev) * 0.2
    outs = {}
    for dt in (torch.float32, torch.bfloat16):
        yy = y.to(dt)
        dst = torch.empty(2, hw, hw, c, device=dev, dtype=dt)
        nt, tp = hip.igemm_bn_bwd_tiles(nhwc(dy.to(dt)), hw, hw, 1, TAPS_3X3, wd, c, nhwc(dst))
        assert nt > 0
        rec = torch.empty(c * nt * 2, device=dev)
        _conv(dy.to(dt), wd, c, dst=dst, bn_bwd=(yy, 1, mu, iv, sc, sh, rec))
        outs[dt] = (dst, rec.view(c, nt, 2), tp)
    same_rounded(outs[torch.bfloat16][0], outs[torch.float32][0], 'data grad')
    g16, rec16, _ = outs[torch.bfloat16]
    g = g16.double().reshape(-1, c)
    yd = y.double().reshape(-1, c)
    dz = torch.where(yd * sc.double() + sh.double() > 0, g, torch.zeros_like(g))  # fma: exact in double
    xhat = (yd - mu.double()) * iv.double()
    # the tiles' sums over the stored (bf16) gradient, totalled per channel
    assert rel(rec16[..., 0].double().sum(1), dz.sum(0)) < 1e-5
    assert rel(rec16[..., 1].double().sum(1), (dz * xhat).sum(0)) < 1e-5


def test_input_layer_forward(dev):
    """The 16-channel input layer (igemm_halo16_c16): 5 bands padded to 16."""
    x = torch.zeros(2, 64, 64, 16, device=dev)
    x[..., :5] = r16(torch.rand(2, 64, 64, 5, device=dev))
    w = torch.randn(64, 5, 3, 3, device=dev) / 45 ** 0.5
    wpk = hip.pack_conv3x3(w, 0, ci_pad=16)
    b = torch.randn(64, device=dev) * 0.1
    y32, _ = _conv(x, wpk, 64, b)
    y16, _ = _conv(x.to(torch.bfloat16), wpk, 64, b, stat=True)
    same_rounded(y16, y32, 'input layer fwd')


@pytest.mark.parametrize('cin,cout', [(128, 64), (512, 512), (64, 64)])
def test_convT_forward_and_data_grad(dev, cin, cout):
    """ConvTranspose2d(k=2, s=2) on the gather16 kernel: the pixel-shuffle forward into a concat slice, the 4-tap
    stride-2 data grad."""
    hc = 16
    x = randn(2, hc, hc, cin, dev=dev, seed=4)
    wT = torch.randn(cin, cout, 2, 2, device=dev) / cin ** 0.5
    bT = torch.randn(cout, device=dev) * 0.1
    wf, wd = hip.pack_convT2x2(wT, 0), hip.pack_convT2x2(wT, 1)
    g = randn(2, 2 * hc, 2 * hc, cout, dev=dev, seed=5)
    res = {}
    for dt in (torch.float32, torch.bfloat16):
        cat = torch.zeros(2, 2 * hc, 2 * hc, cout + 32, device=dev, dtype=dt)
        hip.conv_igemm(nhwc(x.to(dt)), hc, hc, 1, TAPS_1, wf, 4 * cout, bT, nhwc(cat, 32, cout), store_mode=1)
        gx = torch.empty(2, hc, hc, cin, device=dev, dtype=dt)
        hip.conv_igemm(nhwc(g.to(dt)), hc, hc, 2, TAPS_2X2, wd, cin, None, nhwc(gx))
        res[dt] = (cat, gx)
    assert hip.igemm_arith(nhwc(x.to(torch.bfloat16)), hc, hc, 1, TAPS_1, wf, 4 * cout,
                           nhwc(res[torch.bfloat16][0], 32, cout), 1) == 'bf16'
    same_rounded(res[torch.bfloat16][0], res[torch.float32][0], 'ConvT fwd')
    same_rounded(res[torch.bfloat16][1], res[torch.float32][1], 'ConvT data grad')


def _wgrad(dy, x, weight, src_bn=None, rows_bn=None):
    return engine._wgrad3x3(dy, x, weight, src_bn, rows_bn=rows_bn)


@pytest.mark.parametrize('r,c,hw', [(64, 64, 32), (128, 256, 16), (128, 64, 32)])
def test_weight_grad(dev, r, c, hw):
    """The halo weight grad, with and without the source's BatchNorm + ReLU formed while staging: identical slabs."""
    dy = randn(2, hw, hw, r, dev=dev, seed=6)
    x = randn(2, hw, hw, c, dev=dev, seed=7)
    weight = torch.empty(r, c, 3, 3, device=dev)
    sc, sh = torch.rand(2 * c, device=dev) + 0.5, torch.randn(2 * c, device=dev) * 0.3
    for src_bn in (None, (sc, sh, 2)):
        g32 = _wgrad(dy, x, weight, src_bn)
        g16 = _wgrad(dy.to(torch.bfloat16), x.to(torch.bfloat16), weight, src_bn)
        assert torch.equal(g16, g32), src_bn is not None


def test_input_layer_weight_grad_with_rows_bn(dev):
    """The input layer's weight grad forming dy = BN-backward(da, y) while staging (rows_bn), both storages."""
    c, hw = 64, 64
    x = torch.zeros(2, hw, hw, 16, device=dev)
    x[..., :5] = r16(torch.rand(2, hw, hw, 5, device=dev))
    da = randn(2, hw, hw, c, dev=dev, seed=8)
    y = randn(2, hw, hw, c, dev=dev, seed=9)
    mu, iv = torch.randn(2 * c, device=dev) * 0.1, torch.rand(2 * c, device=dev) + 0.5
    sc, sh = torch.rand(2 * c, device=dev) + 0.5, torch.randn(2 * c, device=dev) * 0.2
    gamma = torch.rand(c, device=dev) + 0.5
    coef = torch.randn(2 * c * 2, device=dev) * 0.01
    weight = torch.empty(c, 5, 3, 3, device=dev)
    out = {}
    for dt in (torch.float32, torch.bfloat16):
        assert hip.wgrad_rows_bn_supported(nhwc(da.to(dt)), nhwc(x.to(dt)), 1, TAPS_3X3)
        rows_bn = (nhwc(y.to(dt)), 2, mu, iv, gamma, sc, sh, coef)
        out[dt] = _wgrad(da.to(dt), x.to(dt), weight, rows_bn=rows_bn)
    # dy is formed in fp32 and rounded to bf16 before the product (the bf16 operand) in both storages
    assert torch.equal(out[torch.bfloat16], out[torch.float32])


def test_convT_weight_grad_and_bias(dev):
    cin, cout, hc = 128, 64, 16
    x = randn(2, hc, hc, cin, dev=dev, seed=10)
    g = randn(2, 2 * hc, 2 * hc, cout + 32, dev=dev, seed=11)
    res = {}
    for dt in (torch.float32, torch.bfloat16):
        gv = nhwc(g.to(dt), 32, cout)
        d, ns, nb = hip.wgrad_plan(nhwc(x.to(dt)), gv, 2, TAPS_2X2)
        assert hip.wgrad_arith(d) == 'bf16'
        slabs = torch.empty(nb // 4, device=dev)
        hip.conv_wgrad(d, slabs)
        gw = torch.empty(cin, cout, 2, 2, device=dev)
        hip.wgrad_finalize(slabs, ns, cin, 4, cout, 1, cout, gw)
        gb = torch.empty(cout, device=dev)
        hip.channel_sum(gv, gb, torch.empty(hip.bn_workspace_bytes(2, 2 * hc, 2 * hc, cout, 1), device=dev,
                                            dtype=torch.uint8))
        res[dt] = (gw, gb)
    assert torch.equal(res[torch.bfloat16][0], res[torch.float32][0])
    assert torch.equal(res[torch.bfloat16][1], res[torch.float32][1])


def _bn_stats(y, nseg):
    n, h, w, c = y.shape
    st = [torch.empty(nseg * c, device=y.device) for _ in range(4)]
    ws = torch.empty(hip.bn_workspace_bytes(n, h, w, c, nseg), device=y.device, dtype=torch.uint8)
    gamma, beta = torch.linspace(0.5, 1.5, c, device=y.device), torch.linspace(-0.2, 0.2, c, device=y.device)
    rm, rv = torch.zeros(c, device=y.device), torch.ones(c, device=y.device)
    hip.bn_train_stats(nhwc(y), nseg, gamma, beta, 1e-5, 0.1, True, rm, rv, *st, ws)
    return st, gamma, rm, rv


def test_batchnorm_forward(dev):
    y = randn(4, 32, 32, 128, dev=dev, seed=12)
    s32, _, rm32, rv32 = _bn_stats(y, 2)
    s16, _, rm16, rv16 = _bn_stats(y.to(torch.bfloat16), 2)
    for a, b in zip(s16 + [rm16, rv16], s32 + [rm32, rv32]):
        assert torch.equal(a, b)
    a32 = torch.empty_like(y)
    a16 = torch.empty_like(y, dtype=torch.bfloat16)
    hip.bn_relu_apply(nhwc(y), 2, s32[2], s32[3], nhwc(a32))
    hip.bn_relu_apply(nhwc(y.to(torch.bfloat16)), 2, s32[2], s32[3], nhwc(a16))
    same_rounded(a16, a32, 'bn_relu_apply')


def _bn_bwd_all(y, da, st, gamma, nseg, kind, extra=None):
    n, h, w, c = y.shape
    smean, sinv, scale, shift = st
    dy = torch.empty_like(y)
    dg, db, dbias = (torch.empty(c, device=y.device) for _ in range(3))
    ws = torch.empty(hip.bn_workspace_bytes(n, h, w, c, nseg), device=y.device, dtype=torch.uint8)
    if kind == 'plain':
        hip.bn_relu_backward(nhwc(y), nhwc(da), nseg, smean, sinv, gamma, scale, shift, dg, db, dbias, nhwc(dy), ws)
    elif kind == 'pooled':
        gy, idx, gskip = extra
        hip.bn_relu_backward_pooled(nhwc(y), nhwc(gy), idx, nhwc(gskip), 1, nseg, smean, sinv, gamma, scale, shift,
                                    dg, db, dbias, nhwc(dy), ws)
    else:  # head
        gout, w2 = extra
        hip.bn_relu_backward_head(nhwc(y), gout, w2, w2.shape[0], nseg, smean, sinv, gamma, scale, shift, dg, db,
                                  dbias, nhwc(dy), ws)
    return dy, dg, db, dbias


@pytest.mark.parametrize('kind', ['plain', 'pooled', 'head'])
def test_batchnorm_backward(dev, kind):
    """dy rounded once; dgamma / dbeta bit-identical (same fp32 sums of the same values); the conv-bias sum is the sum
    of the stored dy."""
    n, hw, c = 4, 32, 64
    y = randn(n, hw, hw, c, dev=dev, seed=13)
    st, gamma, _, _ = _bn_stats(y, 2)
    da = randn(n, hw, hw, c, dev=dev, seed=14)
    extra = None
    if kind == 'pooled':  # the Siamese encoder level: pooled gradient through argmax bytes -/+ the difference gradient
        a = torch.empty_like(y)
        hip.bn_relu_apply(nhwc(y), 2, st[2], st[3], nhwc(a))
        pooled = torch.empty(n, hw // 2, hw // 2, c, device=dev)
        idx = torch.empty(n, hw // 2, hw // 2, c, device=dev, dtype=torch.uint8)
        hip.maxpool2_fwd(nhwc(a), nhwc(pooled), idx)
        gy = randn(n, hw // 2, hw // 2, c, dev=dev, seed=15)
        gskip = randn(n // 2, hw, hw, c, dev=dev, seed=16)
        extra32, extra16 = (gy, idx, gskip), (gy.to(torch.bfloat16), idx, gskip.to(torch.bfloat16))
    elif kind == 'head':
        gout = torch.randn(n, 1, hw, hw, device=dev)
        w2 = torch.randn(1, c, device=dev)
        extra32 = extra16 = (gout, w2)
    else:
        extra32 = extra16 = None
    r32 = _bn_bwd_all(y, da, st, gamma, 2, kind, extra32)
    r16_ = _bn_bwd_all(y.to(torch.bfloat16), da.to(torch.bfloat16), st, gamma, 2, kind, extra16)
    same_rounded(r16_[0], r32[0], f'bn backward ({kind}) dy')
    assert torch.equal(r16_[1], r32[1]) and torch.equal(r16_[2], r32[2])
    ref_bias = r16_[0].double().reshape(-1, c).sum(0)
    assert (r16_[3].double() - ref_bias).abs().max().item() <= 1e-5 * ref_bias.abs().max().item() + 1e-4


def test_batchnorm_backward_tiles_and_coef(dev):
    n, hw, c = 2, 32, 64
    y = randn(n, hw, hw, c, dev=dev, seed=17)
    st, gamma, _, _ = _bn_stats(y, 1)
    smean, sinv, scale, shift = st
    da = randn(n, hw, hw, c, dev=dev, seed=18)
    ntiles = n * hw * hw // 128
    rec = torch.randn(c, ntiles, 2, device=dev) * 0.01
    out = {}
    for dt in (torch.float32, torch.bfloat16):
        yy, dd = y.to(dt), da.to(dt)
        dy = torch.empty_like(yy)
        dg, db = torch.empty(c, device=dev), torch.empty(c, device=dev)
        ws = torch.empty(hip.bn_workspace_bytes(n, hw, hw, c, 1), device=dev, dtype=torch.uint8)
        hip.bn_relu_backward_tiles(nhwc(yy), nhwc(dd), 1, smean, sinv, gamma, scale, shift, rec, ntiles, dg, db, None,
                                   nhwc(dy), ws)
        coef = torch.empty(2 * c, device=dev)
        dg2, db2 = torch.empty(c, device=dev), torch.empty(c, device=dev)
        hip.bn_relu_backward_coef(nhwc(yy), nhwc(dd), 1, smean, sinv, gamma, scale, shift, None, 0, coef, dg2, db2, None,
                                  ws)
        out[dt] = (dy, dg, db, coef, dg2, db2)
    same_rounded(out[torch.bfloat16][0], out[torch.float32][0], 'bn backward (tiles) dy')
    for a, b in zip(out[torch.bfloat16][1:], out[torch.float32][1:]):
        assert torch.equal(a, b)


def test_pool_and_difference_kernels(dev):
    n, hw, c = 4, 32, 64
    y = randn(n, hw, hw, c, dev=dev, seed=19)
    st, _, _, _ = _bn_stats(y, 2)
    sc, sh = st[2], st[3]
    res = {}
    for dt in (torch.float32, torch.bfloat16):
        yy = y.to(dt)
        p = torch.empty(n, hw // 2, hw // 2, c, device=dev, dtype=dt)
        i0 = torch.empty(n, hw // 2, hw // 2, c, device=dev, dtype=torch.uint8)
        hip.maxpool2_fwd(nhwc(yy), nhwc(p), i0)
        pb = torch.empty_like(p)
        i1 = torch.empty_like(i0)
        hip.bn_relu_maxpool2_fwd(nhwc(yy), 2, sc, sh, nhwc(pb), i1)
        d = torch.empty(n // 2, hw, hw, c + 16, device=dev, dtype=dt)
        pd = torch.empty_like(p)
        i2 = torch.empty_like(i0)
        hip.bn_relu_pool_diff(nhwc(yy), sc, sh, nhwc(d, 0, c), nhwc(pd), i2)
        d2 = torch.empty(n // 2, hw, hw, c, device=dev, dtype=dt)
        hip.bn_relu_siamese_diff(nhwc(yy), sc, sh, nhwc(d2))
        d3 = torch.empty_like(d2)
        hip.siamese_diff(nhwc(yy), nhwc(d3))
        gx = torch.empty_like(yy)
        hip.feature_grad(nhwc(p), i0, nhwc(d2), 1, nhwc(gx))
        wc = torch.empty(n, hw + 3, hw + 5, c, device=dev, dtype=dt)
        hip.window_copy(nhwc(yy), nhwc(wc), -1, -2)
        res[dt] = dict(p=p, i0=i0, pb=pb, i1=i1, d=d[..., :c], pd=pd, i2=i2, d2=d2, d3=d3, gx=gx, wc=wc)
    a, b = res[torch.bfloat16], res[torch.float32]
    # the feature grad's fp32 twin reads the bf16 run's (rounded) gradients: its output is then one rounding away
    gx = torch.empty_like(y)
    hip.feature_grad(nhwc(a['p'].float()), a['i0'], nhwc(a['d2'].float()), 1, nhwc(gx))
    b['gx'] = gx
    for k in ('i0', 'i1', 'i2'):
        assert torch.equal(a[k], b[k]), k
    for k in ('p', 'pb', 'd', 'pd', 'd2', 'd3', 'gx', 'wc'):
        same_rounded(a[k].contiguous(), b[k].contiguous(), k)


def test_input_pack_and_head(dev):
    n, c, hw = 2, 5, 64
    src = torch.rand(n, c, hw, hw, device=dev)
    p32 = torch.empty(n, hw, hw, 16, device=dev)
    p16 = torch.empty(n, hw, hw, 16, device=dev, dtype=torch.bfloat16)
    hip.pack_nchw(src, 0, c, p32)
    hip.pack_nchw(src, 0, c, p16)
    same_rounded(p16, p32, 'pack_nchw')
    # the 1x1 head: fp32 logits / parameter grads, a bf16 input gradient
    x = randn(n, hw, hw, 64, dev=dev, seed=20)
    w2 = torch.randn(2, 64, device=dev)
    b2 = torch.randn(2, device=dev)
    gout = torch.randn(n, 2, hw, hw, device=dev)
    st, _, _, _ = _bn_stats(x, 1)
    res = {}
    for dt in (torch.float32, torch.bfloat16):
        xx = x.to(dt)
        out = torch.empty(n, 2, hw, hw, device=dev)
        hip.conv1x1_fwd(nhwc(xx), w2, b2, 2, out)
        outb = torch.empty_like(out)
        hip.conv1x1_fwd_bn(nhwc(xx), st[2], st[3], 1, w2, b2, 2, outb)
        gx = torch.empty_like(xx)
        gw, gb = torch.empty(2, 64, device=dev), torch.empty(2, device=dev)
        ws = torch.empty(hip.conv1x1_workspace_bytes(nhwc(xx), 2), device=dev, dtype=torch.uint8)
        hip.conv1x1_bwd(nhwc(xx), w2, gout, 2, nhwc(gx), False, gw, gb, ws)
        gwb, gbb = torch.empty_like(gw), torch.empty_like(gb)
        hip.conv1x1_bwd_bn(nhwc(xx), st[2], st[3], 1, w2, gout, 2, gwb, gbb, ws)
        res[dt] = (out, outb, gx, gw, gb, gwb, gbb)
    a, b = res[torch.bfloat16], res[torch.float32]
    same_rounded(a[2], b[2], 'head input gradient')
    for k in (0, 1, 3, 4, 5, 6):
        assert torch.equal(a[k], b[k]), k


def test_bf16_views_are_refused_outside_the_bf16_kernels(dev):
    """bf16 views need the bf16 arithmetic, and one element type per call."""
    x = torch.zeros(1, 16, 16, 64, device=dev, dtype=torch.bfloat16)
    w = torch.randn(64, 64, 3, 3, device=dev)
    y = torch.empty(1, 16, 16, 64, device=dev, dtype=torch.bfloat16)
    with hip.conv_scope('x3'):
        wpk = hip.pack_conv3x3(w, 0)
        with pytest.raises(RuntimeError, match='bf16 views need math'):
            hip.conv_igemm(nhwc(x), 16, 16, 1, TAPS_3X3, wpk, 64, None, nhwc(y))
    with pytest.raises(RuntimeError, match='different element types'):
        hip.siamese_diff(nhwc(torch.zeros(2, 8, 8, 64, device=dev)), nhwc(torch.empty(1, 8, 8, 64, device=dev,
                                                                                        dtype=torch.bfloat16)))


def test_bf16_models_store_bf16_activations(dev):
    """The bf16 configs' models keep activations and gradients in bf16 (engine.act_storage_for); the h2 default and
    tiles the bf16 kernels do not tile keep fp32."""
    from multimodal_siamese_cd_amd import trainers
    from multimodal_siamese_cd_amd.utils import datasets, experiment_manager as em, networks
    cfg = em.load_cfg('baseline_dualstream')
    net = networks.create_network(cfg).to(dev).train()
    assert net.module.act_storage == torch.bfloat16
    assert networks.create_network(em.load_cfg('baseline_siamese')).module.act_storage == torch.float32
    seen = []
    orig = hip.conv_igemm

    def spy(src, *a, **k):
        seen.append(src.dtype)
        return orig(src, *a, **k)

    hip.conv_igemm = spy
    try:
        gen = torch.Generator(device=dev).manual_seed(1)
        b = datasets.synthetic_batch(cfg, 2, dev, gen, 256)  # deepest level 16 x 16
        loss = trainers.step_loss(cfg, net(b['x_t1'], b['x_t2']), b, net)
        loss.backward()
        assert torch.isfinite(loss)
        assert seen and all(d == hip.DT_BF16 for d in seen), seen
        seen.clear()
        with torch.no_grad():
            net.eval()
            net(b['x_t1'][:, :, :128, :128].contiguous(), b['x_t2'][:, :, :128, :128].contiguous())
        assert seen and all(d == hip.DT_F32 for d in seen)  # deepest level 8 x 8, not tiled: fp32 storage
    finally:
        hip.conv_igemm = orig


@pytest.mark.parametrize('st', [torch.bfloat16, torch.float32])
@pytest.mark.parametrize('ci,co,mode', [(64, 64, 'stats'), (128, 128, 'stats'), (64, 128, 'bn_bwd'), (64, 64, 'in_bn'),
                                        (256, 64, 'plain')])
def test_bf16_1xn_tiles_bit_identical(dev, st, ci, co, mode):
    """The bf16 arithmetic on the 1 x N wave tiles against its 2 x 2 tiles (SCD_TUNE_BF16_1XN flips the layout), both on 128-pixel tiles
    (SCD_TUNE_H2_TILE64_128): every output accumulates the same products in the same order and the epilogue reduces
    in 64-pixel groups in both, so outputs and statistics / BatchNorm-backward records are bit-identical (bf16 and
    fp32 storage)."""
    n, h, w, nseg = 4, 32, 32, 2
    g = torch.Generator(device=dev).manual_seed(ci + co + 3)
    x = torch.randn(n, h, w, ci, device=dev, generator=g).to(st)
    outs = []
    for tune in (hip.TUNE_H2_TILE64_128, hip.TUNE_H2_TILE64_128 | hip.TUNE_BF16_1XN):
        with hip.conv_scope('bf16', tune=tune):
            gw = torch.Generator(device=dev).manual_seed(ci * co)
            wpk = hip.pack_conv3x3(torch.randn(co, ci, 3, 3, device=dev, generator=gw) / (3 * ci ** 0.5), 0)
            sc = torch.rand(nseg * ci, device=dev, generator=gw) + 0.5
            sh = torch.randn(nseg * ci, device=dev, generator=gw) * 0.1
            yb = torch.randn(n, h, w, co, device=dev, generator=gw).to(st)
            mu = torch.randn(nseg * co, device=dev, generator=gw) * 0.1
            iv = torch.rand(nseg * co, device=dev, generator=gw) + .5
            bsc = torch.rand(nseg * co, device=dev, generator=gw) + 0.5
            bsh = torch.randn(nseg * co, device=dev, generator=gw)
            y = torch.full((n, h, w, co), 7.0, device=dev).to(st)
            extra, rec = {}, None
            if mode == 'in_bn':
                extra['in_bn'] = (sc, sh, nseg)
            elif mode == 'stats':
                nt, _ = hip.igemm_stat_tiles(nhwc(x), h, w, 1, hip.TAPS_3X3, wpk, co, nhwc(y))
                rec = extra['stat_rec'] = torch.full((nt * co * 2,), 9.0, device=dev)
            elif mode == 'bn_bwd':
                nt, _ = hip.igemm_bn_bwd_tiles(nhwc(x), h, w, 1, hip.TAPS_3X3, wpk, co, nhwc(y))
                rec = torch.full((co * nt * 2,), 9.0, device=dev)
                extra['bn_bwd'] = (yb, nseg, mu, iv, bsc, bsh, rec)
            assert hip.igemm_arith(nhwc(x), h, w, 1, hip.TAPS_3X3, wpk, co, nhwc(y)) == 'bf16'
            hip.conv_igemm(nhwc(x), h, w, 1, hip.TAPS_3X3, wpk, co, None, nhwc(y), **extra)
            outs.append((y.cpu(), None if rec is None else rec.cpu()))
    assert torch.equal(outs[0][0], outs[1][0])
    if outs[0][1] is not None:
        assert torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize('mode', ['stats', 'bn_bwd', 'plain'])
def test_bf16_tn4_tile_bit_identical(dev, mode):
    """the 128 x 256 bf16 block (1 x 4 waves of 128 px x 64 ch, the automatic choice for >= 256 outputs on
    grids of >= 512 such blocks) against the 128 x 128 1 x 4 tile (SCD_TUNE_HALO16_CFG(3)) and the 2 x 2 tile
    (SCD_TUNE_BF16_1XN flip): same products in the same order and 64-pixel reduction groups, so outputs and
    statistics / BatchNorm-backward records are bit-identical.  256 -> 256 channels at 16 x 64 x 64 = 512 blocks."""
    n, h, w, ci, co, nseg = 16, 64, 64, 256, 256, 2
    assert n * h * w // 128 * (co // 256) >= 512
    g = torch.Generator(device=dev).manual_seed(11)
    x = torch.randn(n, h, w, ci, device=dev, generator=g).to(torch.bfloat16)
    outs = []
    for tune in (0, hip.tune_halo16_cfg(3), hip.TUNE_BF16_1XN):
        with hip.conv_scope('bf16', tune=tune):
            gw = torch.Generator(device=dev).manual_seed(5)
            wpk = hip.pack_conv3x3(torch.randn(co, ci, 3, 3, device=dev, generator=gw) / (3 * ci ** 0.5), 0)
            yb = torch.randn(n, h, w, co, device=dev, generator=gw).to(torch.bfloat16)
            mu = torch.randn(nseg * co, device=dev, generator=gw) * 0.1
            iv = torch.rand(nseg * co, device=dev, generator=gw) + .5
            bsc = torch.rand(nseg * co, device=dev, generator=gw) + 0.5
            bsh = torch.randn(nseg * co, device=dev, generator=gw)
            y = torch.full((n, h, w, co), 7.0, device=dev).to(torch.bfloat16)
            extra, rec = {}, None
            if mode == 'stats':
                nt, _ = hip.igemm_stat_tiles(nhwc(x), h, w, 1, hip.TAPS_3X3, wpk, co, nhwc(y))
                rec = extra['stat_rec'] = torch.full((nt * co * 2,), 9.0, device=dev)
            elif mode == 'bn_bwd':
                nt, _ = hip.igemm_bn_bwd_tiles(nhwc(x), h, w, 1, hip.TAPS_3X3, wpk, co, nhwc(y))
                rec = torch.full((co * nt * 2,), 9.0, device=dev)
                extra['bn_bwd'] = (yb, nseg, mu, iv, bsc, bsh, rec)
            assert hip.igemm_arith(nhwc(x), h, w, 1, hip.TAPS_3X3, wpk, co, nhwc(y)) == 'bf16'
            hip.conv_igemm(nhwc(x), h, w, 1, hip.TAPS_3X3, wpk, co, None, nhwc(y), **extra)
            outs.append((y.cpu(), None if rec is None else rec.cpu()))
    for o in outs[1:]:
        assert torch.equal(outs[0][0], o[0])
        if outs[0][1] is not None:
            assert torch.equal(outs[0][1], o[1])


@pytest.mark.parametrize('src_bn', [False, True])
@pytest.mark.parametrize('n,h,w,r,c,cs', [(4, 32, 32, 128, 64, 0), (3, 16, 48, 64, 128, 32), (2, 2, 16, 128, 128, 0),
                                          (9, 8, 64, 256, 64, 64), (1, 64, 16, 64, 64, 0)])
def test_weight_grad_dma_ring_bit_identical(dev, n, h, w, r, c, cs, src_bn):
    """The bf16-storage halo weight grad with its patches brought in by LDS-DMA (the default) against the
    register-staged kernel (SCD_TUNE_WGRAD16_REGSTAGE): identical split plan, every slab element written
    (NaN-prefilled) and bit-identical; 128-row (8-wave) and 64-row blocks, image borders on every side (zero halo from
    out-of-range DMA pieces), one patch row (h = 2), splits shorter than the ring, channel slices of wider buffers (the
    decoder's concat views: ldc > c), and the source read through its BatchNorm + ReLU (two segments, transformed in
    LDS one patch ahead: negative shifts make the zero padding differ from relu(shift))."""
    g = torch.Generator(device=dev).manual_seed(n * h + w + r + c)
    dyb = torch.randn(n, h, w, cs + r, device=dev, generator=g).to(torch.bfloat16)
    xb = torch.randn(n, h, w, c + cs, device=dev, generator=g).to(torch.bfloat16)
    rows, src = nhwc(dyb, cs, r), nhwc(xb, 0, c)
    bn = None
    if src_bn:
        nseg = 2 if n % 2 == 0 else 1
        bn = (torch.rand(nseg * c, device=dev, generator=g) + 0.5, torch.randn(nseg * c, device=dev, generator=g) * 0.5,
              nseg)
    out = []
    for tune in (0, hip.TUNE_WGRAD16_REGSTAGE):
        with hip.conv_scope('bf16', tune=tune):
            d, nsplit, nbytes = hip.wgrad_plan(rows, src, 1, TAPS_3X3, bn)
            assert hip.wgrad_arith(d) == 'bf16'
            slabs = torch.full((nbytes // 4,), float('nan'), device=dev)
            hip.conv_wgrad(d, slabs)
            out.append((nsplit, slabs.cpu()))
    assert out[0][0] == out[1][0]
    assert not torch.isnan(out[0][1]).any()
    assert torch.equal(out[0][1], out[1][1])


@pytest.mark.parametrize('n,h,w,r,c,nseg,src_bn', [(4, 32, 32, 128, 64, 2, False), (2, 16, 48, 64, 128, 2, True),
                                                   (3, 8, 32, 256, 64, 1, True), (2, 2, 16, 64, 64, 1, False)])
def test_weight_grad_dma_ring_rows_bn_bit_identical(dev, n, h, w, r, c, nseg, src_bn):
    """The DMA-ring weight grad forming a plain BatchNorm backward's dY in LDS (y and dL/da landed raw, ABI 8 rows_bn)
    against the register-staged kernel: the stored dY (rows_out, written once by the channel-tile-0 blocks), its bound
    and every slab element bit-identical, with and without the source transform, 64- and 128-row blocks, two row tiles
    (r = 256), one patch row."""
    g = torch.Generator(device=dev).manual_seed(n + h + w + r + c)
    da = torch.randn(n, h, w, r, device=dev, generator=g).to(torch.bfloat16)
    y = (torch.randn(n, h, w, r, device=dev, generator=g) * 2 + 0.3).to(torch.bfloat16)
    x = torch.randn(n, h, w, c, device=dev, generator=g).to(torch.bfloat16)
    mu, iv = torch.randn(nseg * r, device=dev, generator=g) * 0.1, torch.rand(nseg * r, device=dev, generator=g) + .5
    sc, sh = torch.rand(nseg * r, device=dev, generator=g) + 0.5, torch.randn(nseg * r, device=dev, generator=g) * 0.3
    gamma = torch.rand(r, device=dev, generator=g) + 0.5
    coef = torch.randn(nseg * r * 2, device=dev, generator=g) * 0.01
    xbn = ((torch.rand(nseg * c, device=dev, generator=g) + 0.5, torch.randn(nseg * c, device=dev, generator=g) * 0.5,
            nseg) if src_bn else None)
    out = []
    for tune in (0, hip.TUNE_WGRAD16_REGSTAGE):
        with hip.conv_scope('bf16', tune=tune):
            assert hip.wgrad_rows_bn_supported(nhwc(da), nhwc(x), 1, TAPS_3X3, xbn)
            dy = torch.full_like(y, float('nan'))
            bound = torch.zeros(1, device=dev)
            d, nsplit, nbytes = hip.wgrad_plan(nhwc(da), nhwc(x), 1, TAPS_3X3, xbn,
                                               rows_bn=(nhwc(y), nseg, mu, iv, gamma, sc, sh, coef), rows_out=nhwc(dy),
                                               rows_out_bound=bound)
            slabs = torch.full((nbytes // 4,), float('nan'), device=dev)
            hip.conv_wgrad(d, slabs)
            out.append((nsplit, slabs.cpu(), dy.cpu(), bound.item()))
    assert out[0][0] == out[1][0]
    assert not torch.isnan(out[0][1]).any() and not torch.isnan(out[0][2].float()).any()
    assert torch.equal(out[0][1], out[1][1])
    assert torch.equal(out[0][2], out[1][2])
    assert out[0][3] == out[1][3] == out[0][2].float().abs().max().item()
