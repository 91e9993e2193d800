"""Per-kernel parity on MI355X: each libscd entry point vs the torch fp32 CPU op it replaces.

Tolerance: max|hip - ref| / max|ref| <= 1e-5 for single ops; argmax indices are bit-exact.
- fp32 MFMA is exact fp32 fmaf chains, so the residual is summation order only.
- The split-bf16 x3 conv math drops only terms of <= ~2^-26 relative size.
Every conv test runs under both conv arithmetics (scd_set_conv_math).
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import siamese_oracle as O

pytestmark = pytest.mark.gpu

TOL = 1e-5


@pytest.fixture(scope='module')
def dev():
    from multimodal_siamese_cd_amd import hip
    hip.load_library()
    d = torch.device('cuda:0')
    hip.ensure_device(torch.empty(1, device=d))
    return d


@pytest.fixture(params=['f32', 'x3'])
def math(request, dev):
    from multimodal_siamese_cd_amd import hip
    prev = hip.set_conv_math(request.param)
    yield request.param
    hip.set_conv_math(prev)


def rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


def nchw(t):
    return t.permute(0, 3, 1, 2).contiguous()


def nhwc_t(t):
    return t.permute(0, 2, 3, 1).contiguous()


CONV_SHAPES = [  # n, h, w, cin, cout
    (2, 16, 16, 8, 8),
    (2, 9, 13, 16, 40),
    (1, 8, 8, 64, 128),
    (2, 32, 32, 128, 64),
    (3, 5, 7, 24, 200),
    (2, 16, 16, 512, 512),
]


@pytest.mark.parametrize('n,h,w,ci,co', CONV_SHAPES)
def test_conv3x3_forward(dev, math, n, h, w, ci, co):
    from multimodal_siamese_cd_amd import hip
    g = torch.Generator().manual_seed(n * 1000 + ci + co)
    x = torch.randn(n, h, w, ci, generator=g)
    wt = torch.randn(co, ci, 3, 3, generator=g) / (3 * ci ** 0.5)
    b = torch.randn(co, generator=g)
    ref = nhwc_t(F.conv2d(nchw(x), wt, b, padding=1))
    xd, wd, bd = x.to(dev), wt.to(dev), b.to(dev)
    y = torch.empty(n, h, w, co, device=dev)
    hip.conv_igemm(hip.nhwc(xd), h, w, 1, hip.TAPS_3X3, hip.pack_conv3x3(wd, 0), co, bd, hip.nhwc(y))
    assert rel(y, ref) < TOL


@pytest.mark.parametrize('n,h,w,ci,co', CONV_SHAPES)
def test_conv3x3_data_and_weight_grad(dev, math, n, h, w, ci, co):
    from multimodal_siamese_cd_amd import hip
    g = torch.Generator().manual_seed(7 + n + ci * co)
    x = torch.randn(n, h, w, ci, generator=g)
    wt = torch.randn(co, ci, 3, 3, generator=g) / (3 * ci ** 0.5)
    dy = torch.randn(n, h, w, co, generator=g)
    ref_dx = nhwc_t(torch.nn.grad.conv2d_input((n, ci, h, w), wt, nchw(dy), padding=1))
    ref_dw = torch.nn.grad.conv2d_weight(nchw(x), wt.shape, nchw(dy), padding=1)
    xd, wd, dyd = x.to(dev), wt.to(dev), dy.to(dev)
    dx = torch.empty(n, h, w, ci, device=dev)
    hip.conv_igemm(hip.nhwc(dyd), h, w, 1, hip.TAPS_3X3, hip.pack_conv3x3(wd, 1), ci, None, hip.nhwc(dx))
    assert rel(dx, ref_dx) < TOL
    d, nsplit, nbytes = hip.wgrad_plan(hip.nhwc(dyd), hip.nhwc(xd), 1, hip.TAPS_3X3)
    slabs = torch.empty(nbytes // 4, device=dev)
    hip.conv_wgrad(d, slabs)
    dw = torch.empty(co, ci, 3, 3, device=dev)
    hip.wgrad_finalize(slabs, nsplit, co, 9, ci, 0, ci, dw)
    assert rel(dw, ref_dw) < TOL


def test_conv3x3_channel_padded_input(dev, math):
    """First layer: 5 real input channels padded to 8 in NHWC (zero channels, zero weights)."""
    from multimodal_siamese_cd_amd import hip
    g = torch.Generator().manual_seed(3)
    n, h, w, ci, co = 2, 12, 20, 5, 16
    x = torch.rand(n, ci, h, w, generator=g)
    wt = torch.randn(co, ci, 3, 3, generator=g)
    b = torch.randn(co, generator=g)
    ref = nhwc_t(F.conv2d(x, wt, b, padding=1))
    xp = torch.empty(n, h, w, 8, device=dev)
    hip.pack_nchw(x.to(dev), 0, ci, xp)
    assert torch.equal(xp[..., 5:].cpu(), torch.zeros(n, h, w, 3))
    y = torch.empty(n, h, w, co, device=dev)
    hip.conv_igemm(hip.nhwc(xp), h, w, 1, hip.TAPS_3X3, hip.pack_conv3x3(wt.to(dev), 0, ci_pad=8), co, b.to(dev),
                   hip.nhwc(y))
    assert rel(y, ref) < TOL
    dy = torch.randn(n, h, w, co, generator=g)
    ref_dw = torch.nn.grad.conv2d_weight(x, wt.shape, nchw(dy), padding=1)
    d, nsplit, nbytes = hip.wgrad_plan(hip.nhwc(dy.to(dev)), hip.nhwc(xp), 1, hip.TAPS_3X3)
    slabs = torch.empty(nbytes // 4, device=dev)
    hip.conv_wgrad(d, slabs)
    dw = torch.empty(co, ci, 3, 3, device=dev)
    hip.wgrad_finalize(slabs, nsplit, co, 9, 8, 0, ci, dw)
    assert rel(dw, ref_dw) < TOL


@pytest.mark.parametrize('ci,co', [(64, 128), (512, 512), (128, 64)])
def test_conv_math_accuracy_vs_fp64(dev, ci, co):
    """Both arithmetics against an fp64 conv on wide-dynamic-range data (magnitudes spread over 1e-3..1e3).

    The x3 split must be as accurate as fp32 MFMA: its error may not exceed 2x the fp32 kernel's error,
    and both must stay at fp32 rounding level.
    """
    from multimodal_siamese_cd_amd import hip
    g = torch.Generator().manual_seed(ci + 3 * co)
    n, h, w = 2, 24, 20
    x = torch.randn(n, h, w, ci, generator=g, dtype=torch.float64) * 10 ** (6 * torch.rand(n, h, w, ci, generator=g, dtype=torch.float64) - 3)
    wt = torch.randn(co, ci, 3, 3, generator=g, dtype=torch.float64) / (3 * ci ** 0.5)
    x, wt = x.float(), wt.float()
    ref = nhwc_t(F.conv2d(nchw(x).double(), wt.double(), None, padding=1))
    errs = {}
    for m in ('f32', 'x3', 'x3-onthefly'):
        prev = hip.set_conv_math(m.split('-')[0])
        y = torch.empty(n, h, w, co, device=dev)
        wpk = hip.pack_conv3x3(wt.to(dev), 0)
        if m == 'x3-onthefly':  # weights split inside every workgroup instead of pre-split planes
            del wpk._x3
        hip.conv_igemm(hip.nhwc(x.to(dev)), h, w, 1, hip.TAPS_3X3, wpk, co, None, hip.nhwc(y))
        hip.set_conv_math(prev)
        errs[m] = rel(y, ref)
    assert max(errs.values()) < 1e-5, errs
    assert errs['x3'] <= 2 * errs['f32'] + 1e-7, errs
    assert errs['x3-onthefly'] <= 2 * errs['f32'] + 1e-7, errs


@pytest.mark.parametrize('ci,co', [(64, 64), (128, 256), (8, 64)])
def test_wgrad_math_accuracy_vs_fp64(dev, ci, co):
    """Weight gradient under both arithmetics against fp64, on wide-dynamic-range data.

    Pixels are the K dimension here (long sums), so this also exercises the split-K slab reduction.
    """
    from multimodal_siamese_cd_amd import hip
    g = torch.Generator().manual_seed(5 * ci + co)
    n, h, w = 4, 40, 48  # 2x16 patches: the x3 halo weight-grad path for C, R multiples of 64
    x = (torch.randn(n, h, w, ci, generator=g, dtype=torch.float64)
         * 10 ** (4 * torch.rand(n, h, w, ci, generator=g, dtype=torch.float64) - 2)).float()
    dy = (torch.randn(n, h, w, co, generator=g, dtype=torch.float64)
          * 10 ** (4 * torch.rand(n, h, w, co, generator=g, dtype=torch.float64) - 2)).float()
    ref = torch.nn.grad.conv2d_weight(nchw(x).double(), (co, ci, 3, 3), nchw(dy).double(), padding=1)
    errs = {}
    for m in ('f32', 'x3'):
        prev = hip.set_conv_math(m)
        xd, dyd = x.to(dev), dy.to(dev)
        d, nsplit, nbytes = hip.wgrad_plan(hip.nhwc(dyd), hip.nhwc(xd), 1, hip.TAPS_3X3)
        slabs = torch.empty(nbytes // 4, device=dev)
        hip.conv_wgrad(d, slabs)
        dw = torch.empty(co, ci, 3, 3, device=dev)
        hip.wgrad_finalize(slabs, nsplit, co, 9, ci, 0, ci, dw)
        hip.set_conv_math(prev)
        errs[m] = rel(dw, ref)
    assert max(errs.values()) < 1e-5, errs
    assert errs['x3'] <= 2 * errs['f32'] + 1e-7, errs


@pytest.mark.parametrize('n,h,w,c,cs', [(2, 8, 8, 16, 16), (1, 16, 16, 64, 64), (2, 4, 6, 512, 512), (2, 3, 5, 8, 24)])
def test_convT2x2_forward_into_concat_slice(dev, math, n, h, w, c, cs):
    from multimodal_siamese_cd_amd import hip
    g = torch.Generator().manual_seed(c + h)
    x = torch.randn(n, h, w, c, generator=g)
    wt = torch.randn(c, c, 2, 2, generator=g) / c ** 0.5
    b = torch.randn(c, generator=g)
    ref = nhwc_t(F.conv_transpose2d(nchw(x), wt, b, stride=2))
    cat = torch.full((n, 2 * h, 2 * w, cs + c), float('nan'), device=dev)
    xd, wd, bd = x.to(dev), wt.to(dev), b.to(dev)
    hip.conv_igemm(hip.nhwc(xd), h, w, 1, hip.TAPS_1, hip.pack_convT2x2(wd, 0), 4 * c, bd, hip.nhwc(cat, cs, c),
                   store_mode=1)
    assert rel(cat[..., cs:], ref) < TOL
    assert torch.isnan(cat[..., :cs]).all(), 'wrote outside its channel slice'


@pytest.mark.parametrize('n,h,w,c,cs', [(2, 8, 8, 16, 16), (1, 16, 16, 64, 64), (2, 4, 6, 512, 512)])
def test_convT2x2_backward(dev, math, n, h, w, c, cs):
    from multimodal_siamese_cd_amd import hip
    g = torch.Generator().manual_seed(11 + c)
    x = torch.randn(n, c, h, w, generator=g, requires_grad=True)
    wt = (torch.randn(c, c, 2, 2, generator=g) / c ** 0.5).requires_grad_(True)
    b = torch.randn(c, generator=g, requires_grad=True)
    out = F.conv_transpose2d(x, wt, b, stride=2)
    gy = torch.randn(out.shape, generator=g)
    out.backward(gy)
    gcat = torch.randn(n, 2 * h, 2 * w, cs + c, generator=g)
    gcat[..., cs:] = nhwc_t(gy)
    gd = gcat.to(dev)
    gup = hip.nhwc(gd, cs, c)
    xd = nhwc_t(x.detach()).to(dev)
    gx = torch.empty(n, h, w, c, device=dev)
    hip.conv_igemm(gup, h, w, 2, hip.TAPS_2X2, hip.pack_convT2x2(wt.detach().to(dev), 1), c, None, hip.nhwc(gx))
    assert rel(gx, nhwc_t(x.grad)) < TOL
    d, nsplit, nbytes = hip.wgrad_plan(hip.nhwc(xd), gup, 2, hip.TAPS_2X2)
    slabs = torch.empty(nbytes // 4, device=dev)
    hip.conv_wgrad(d, slabs)
    gw = torch.empty(c, c, 2, 2, device=dev)
    hip.wgrad_finalize(slabs, nsplit, c, 4, c, 1, c, gw)
    assert rel(gw, wt.grad) < TOL
    gb = torch.empty(c, device=dev)
    hip.channel_sum(gup, gb, torch.empty(hip.bn_workspace_bytes(n, 2 * h, 2 * w, c, 1), dtype=torch.uint8, device=dev))
    assert rel(gb, b.grad) < TOL


@pytest.mark.parametrize('arith', ['h2', 'x3', 'bf16'])
@pytest.mark.parametrize('n,h,w,c,cs', [(2, 8, 8, 16, 16), (4, 16, 16, 64, 64), (2, 4, 6, 512, 512), (32, 64, 64, 128, 64)])
def test_convT_bias_grad_from_weight_grad_staging(dev, arith, n, h, w, c, cs):
    """The ConvTranspose bias grad from the weight grad's column sums (scd_wgrad_t.src_colsum, every split's slab
    written: NaN-prefilled) == the float64 sum of dOut over the concat slice, as scd_channel_sum, in each arithmetic
    (bf16: bf16 storage of dOut and x).  The weight grad itself is unchanged by the extra output."""
    from multimodal_siamese_cd_amd import hip
    st = torch.bfloat16 if arith == 'bf16' else torch.float32
    g = torch.Generator().manual_seed(5 + c + n)
    gd = torch.randn(n, 2 * h, 2 * w, cs + c, generator=g).to(dev).to(st)
    xd = torch.randn(n, h, w, c, generator=g).to(dev).to(st)
    gup = hip.nhwc(gd, cs, c)
    with hip.conv_scope(arith):
        bounds = (xd.float().abs().max().reshape(1), gd.float().abs().max().reshape(1)) if arith == 'h2' else (None, None)
        outs = []
        for with_cs in (False, True):
            d, nsplit, nbytes = hip.wgrad_plan(hip.nhwc(xd), gup, 2, hip.TAPS_2X2, None, *bounds)
            assert hip.wgrad_colsum_supported(d)
            colsum = torch.full((nsplit * 4 * c,), float('nan'), device=dev)
            if with_cs:
                d.src_colsum = colsum.data_ptr()
            slabs = torch.empty(nbytes // 4, device=dev)
            hip.conv_wgrad(d, slabs)
            gw = torch.empty(c, c, 2, 2, device=dev)
            hip.wgrad_finalize(slabs, nsplit, c, 4, c, 1, c, gw)
            outs.append(gw)
        assert torch.equal(outs[0], outs[1])
        assert bool(torch.isfinite(colsum).all())
        gb = torch.empty(c, device=dev)
        hip.wgrad_colsum_finalize(colsum, nsplit, 4, c, gb)
    exact = gd[..., cs:].double().sum((0, 1, 2)).cpu()
    scale = gd[..., cs:].double().abs().sum((0, 1, 2)).max().item()
    assert (gb.double().cpu() - exact).abs().max().item() / scale < 1e-6
    ref = torch.empty(c, device=dev)
    hip.channel_sum(gup, ref, torch.empty(hip.bn_workspace_bytes(n, 2 * h, 2 * w, c, 1), dtype=torch.uint8, device=dev))
    assert (ref.double().cpu() - exact).abs().max().item() / scale < 1e-6


def test_convT_bias_colsum_refused_off_the_generic_kernel(dev):
    """A 3x3 weight grad on the halo kernels has no column sums: setting src_colsum there is refused."""
    from multimodal_siamese_cd_amd import hip
    x = torch.randn(2, 16, 16, 64, device=dev)
    dy = torch.randn(2, 16, 16, 64, device=dev)
    with hip.conv_scope('x3'):
        d, nsplit, nbytes = hip.wgrad_plan(hip.nhwc(dy), hip.nhwc(x), 1, hip.TAPS_3X3)
        assert not hip.wgrad_colsum_supported(d)
        colsum = torch.empty(nsplit * 9 * 64, device=dev)
        d.src_colsum = colsum.data_ptr()
        with pytest.raises(RuntimeError, match='src_colsum'):
            hip.conv_wgrad(d, torch.empty(nbytes // 4, device=dev))


@pytest.mark.parametrize('n,h,w,ci,co,nseg', [(4, 32, 32, 64, 128, 2), (4, 16, 16, 32, 64, 2), (2, 64, 64, 16, 32, 1),
                                              (2, 16, 16, 512, 512, 1)])
def test_conv_fused_bn_stats(dev, n, h, w, ci, co, nseg):
    """Conv-fused per-tile BatchNorm statistics (x3 halo path) == the separate statistics pass on the same y."""
    from multimodal_siamese_cd_amd import hip
    prev = hip.set_conv_math('x3')
    try:
        g = torch.Generator().manual_seed(ci * co + n)
        x = torch.randn(n, h, w, ci, generator=g).to(dev)
        wt = (torch.randn(co, ci, 3, 3, generator=g) / (3 * ci ** 0.5)).to(dev)
        b = (torch.randn(co, generator=g) + 3.0).to(dev)  # offset: M2 about a non-zero mean
        wpk = hip.pack_conv3x3(wt, 0)
        y = torch.empty(n, h, w, co, device=dev)
        ntiles, tpx = hip.igemm_stat_tiles(hip.nhwc(x), h, w, 1, hip.TAPS_3X3, wpk, co, hip.nhwc(y))
        assert ntiles > 0 and ntiles * tpx == n * h * w
        rec = torch.empty(ntiles * co * 2, device=dev)
        hip.conv_igemm(hip.nhwc(x), h, w, 1, hip.TAPS_3X3, wpk, co, b, hip.nhwc(y), stat_rec=rec)
        gamma = torch.rand(co, device=dev) + 0.5
        beta = torch.randn(co, device=dev)
        outs = []
        for fused in (False, True):
            rm, rv = torch.zeros(co, device=dev), torch.ones(co, device=dev)
            o = [torch.empty(nseg * co, device=dev) for _ in range(4)]
            if fused:
                ws = torch.empty(hip.bn_tile_stats_workspace_bytes(ntiles, co, nseg), dtype=torch.uint8, device=dev)
                hip.bn_stats_from_tiles(rec, ntiles, tpx, co, nseg, gamma, beta, 1e-5, 0.1, True, rm, rv, *o, ws)
            else:
                ws = torch.empty(hip.bn_workspace_bytes(n, h, w, co, nseg), dtype=torch.uint8, device=dev)
                hip.bn_train_stats(hip.nhwc(y), nseg, gamma, beta, 1e-5, 0.1, True, rm, rv, *o, ws)
            outs.append(o + [rm, rv])
        for a, b_ in zip(*outs):
            assert rel(a, b_) < 2e-6
        # and against the definition on the host
        yc = y.double().cpu().reshape(nseg, -1, co)
        assert rel(outs[1][0].reshape(nseg, co), yc.mean(1)) < 2e-6
        assert rel(outs[1][1].reshape(nseg, co), 1 / torch.sqrt(yc.var(1, unbiased=False) + 1e-5)) < 2e-6
    finally:
        hip.set_conv_math(prev)


HALO16_SHAPES = [  # n, h, w, cin, cout: tile widths 64 / 32 / 16, ragged n_out, 512-channel layers
    (2, 32, 64, 64, 128),
    (2, 16, 32, 128, 128),
    (1, 16, 16, 32, 256),
    (2, 8, 64, 96, 136),
    (2, 16, 16, 512, 512),
]


@pytest.mark.parametrize('cfg', [0, 1, 2])
@pytest.mark.parametrize('n,h,w,ci,co', HALO16_SHAPES)
def test_conv_halo16_tiles(dev, cfg, n, h, w, ci, co):
    """16x16x32-MFMA halo kernel, every tile config forced: forward (+ bias, fused BN tile statistics) and
    data-grad against torch fp32, statistics against the separate pass."""
    from multimodal_siamese_cd_amd import hip
    prev_m = hip.set_conv_math('x3')
    prev_h = hip.set_halo16(2 + cfg)
    try:
        g = torch.Generator().manual_seed(11 * cfg + ci + co)
        x = torch.randn(n, h, w, ci, generator=g)
        wt = torch.randn(co, ci, 3, 3, generator=g) / (3 * ci ** 0.5)
        b = torch.randn(co, generator=g) + 2.0
        ref = nhwc_t(F.conv2d(nchw(x), wt, b, padding=1))
        xd, wd, bd = x.to(dev), wt.to(dev), b.to(dev)
        wpk = hip.pack_conv3x3(wd, 0)
        y = torch.empty(n, h, w, co, device=dev)
        ntiles, tpx = hip.igemm_stat_tiles(hip.nhwc(xd), h, w, 1, hip.TAPS_3X3, wpk, co, hip.nhwc(y))
        assert ntiles * tpx == n * h * w and tpx == (128 if cfg < 2 else 64)
        rec = torch.empty(ntiles * co * 2, device=dev)
        hip.conv_igemm(hip.nhwc(xd), h, w, 1, hip.TAPS_3X3, wpk, co, bd, hip.nhwc(y), stat_rec=rec)
        assert rel(y, ref) < TOL
        # per-tile (mean, M2) records against the host definition on the kernel's own output
        tw = next(c for c in (hip.halo16_tile_width_pref(), 64, 32, 16)
                  if w % c == 0 and tpx % c == 0 and h % (tpx // c) == 0)
        tr = tpx // tw
        yy = y.double().cpu().reshape(n, h // tr, tr, w // tw, tw, co).permute(0, 1, 3, 2, 4, 5).reshape(-1, tpx, co)
        r = rec.double().cpu().reshape(ntiles, co, 2)
        assert rel(r[..., 0], yy.mean(1)) < 2e-6
        assert rel(r[..., 1], ((yy - yy.mean(1, keepdim=True)) ** 2).sum(1)) < 2e-5
        # data-grad (n_out = ci)
        if ci % 4 == 0:
            dy = torch.randn(n, h, w, co, generator=g)
            ref_dx = nhwc_t(torch.nn.grad.conv2d_input((n, ci, h, w), wt, nchw(dy), padding=1))
            dx = torch.empty(n, h, w, ci, device=dev)
            hip.conv_igemm(hip.nhwc(dy.to(dev)), h, w, 1, hip.TAPS_3X3, hip.pack_conv3x3(wd, 1), ci, None, hip.nhwc(dx))
            assert rel(dx, ref_dx) < TOL
    finally:
        hip.set_halo16(prev_h)
        hip.set_conv_math(prev_m)


@pytest.mark.parametrize('n,h,w,ci,co,nseg', [(4, 16, 32, 64, 128, 2), (2, 8, 64, 128, 64, 1), (4, 8, 16, 64, 64, 2)])
def test_fused_input_bn(dev, n, h, w, ci, co, nseg):
    """Conv forward and weight grad reading y through BN-apply + ReLU (in_bn / src_bn) are bit-identical to the
    same kernels on the materialised activation (bn_relu_apply), per-segment coefficients included."""
    from multimodal_siamese_cd_amd import hip
    prev_m = hip.set_conv_math('x3')
    try:
        g = torch.Generator().manual_seed(n * h + ci)
        y = torch.randn(n, h, w, ci, generator=g).to(dev)
        sc = (torch.rand(nseg * ci, generator=g) * 2 - 0.5).to(dev)  # some negative scales
        sh = torch.randn(nseg * ci, generator=g).to(dev)
        a = torch.empty_like(y)
        hip.bn_relu_apply(hip.nhwc(y), nseg, sc, sh, hip.nhwc(a))
        wt = (torch.randn(co, ci, 3, 3, generator=g) / (3 * ci ** 0.5)).to(dev)
        b = torch.randn(co, generator=g).to(dev)
        wpk = hip.pack_conv3x3(wt, 0)
        out_ref, out = torch.empty(n, h, w, co, device=dev), torch.empty(n, h, w, co, device=dev)
        bn = (sc, sh, nseg)
        assert hip.igemm_input_bn_supported(hip.nhwc(y), h, w, 1, hip.TAPS_3X3, wpk, co, hip.nhwc(out), bn)
        hip.conv_igemm(hip.nhwc(a), h, w, 1, hip.TAPS_3X3, wpk, co, b, hip.nhwc(out_ref))
        hip.conv_igemm(hip.nhwc(y), h, w, 1, hip.TAPS_3X3, wpk, co, b, hip.nhwc(out), in_bn=bn)
        assert torch.equal(out, out_ref)
        dy = torch.randn(n, h, w, co, generator=g).to(dev)
        dws = []
        for src, sbn in ((a, None), (y, bn)):
            if sbn is not None:
                assert hip.wgrad_src_bn_supported(hip.nhwc(dy), hip.nhwc(y), 1, hip.TAPS_3X3, sbn)
            d, nsplit, nbytes = hip.wgrad_plan(hip.nhwc(dy), hip.nhwc(src), 1, hip.TAPS_3X3, sbn)
            slabs = torch.empty(nbytes // 4, device=dev)
            hip.conv_wgrad(d, slabs)
            dw = torch.empty(co, ci, 3, 3, device=dev)
            hip.wgrad_finalize(slabs, nsplit, co, 9, ci, 0, ci, dw)
            dws.append(dw)
        assert torch.equal(dws[0], dws[1])
        # not offered where the kernel cannot apply it: fp32 arithmetic -> the call is rejected, not ignored
        hip.set_conv_math('f32')
        assert not hip.igemm_input_bn_supported(hip.nhwc(y), h, w, 1, hip.TAPS_3X3, wpk, co, hip.nhwc(out), bn)
        with pytest.raises(RuntimeError):
            hip.conv_igemm(hip.nhwc(y), h, w, 1, hip.TAPS_3X3, wpk, co, b, hip.nhwc(out), in_bn=bn)
    finally:
        hip.set_conv_math(prev_m)


@pytest.mark.parametrize('n,h,w,ci,co,nseg', [(4, 16, 32, 128, 64, 2), (2, 32, 16, 64, 128, 1), (4, 8, 16, 256, 96, 2)])
def test_fused_bn_backward_partials(dev, n, h, w, ci, co, nseg):
    """Data-grad conv with BatchNorm-backward partial sums in its epilogue + bn_relu_backward_tiles == the conv
    followed by bn_relu_backward's own partial pass (dy, dgamma, dbeta, conv-bias grad)."""
    from multimodal_siamese_cd_amd import hip
    prev_m = hip.set_conv_math('x3')
    try:
        g = torch.Generator().manual_seed(n + ci + co)
        dy1 = torch.randn(n, h, w, ci, generator=g).to(dev)  # gradient of the next conv's output (ci channels)
        wt = (torch.randn(ci, co, 3, 3, generator=g) / (3 * ci ** 0.5)).to(dev)  # next conv: co -> ci
        wb = hip.pack_conv3x3(wt, 1)
        y0 = torch.randn(n, h, w, co, generator=g).to(dev)  # BN input (conv output of this layer)
        gamma = (torch.rand(co, generator=g) + 0.5).to(dev)
        beta = torch.randn(co, generator=g).to(dev)
        smean, sinv, scale, shift = (torch.empty(nseg * co, device=dev) for _ in range(4))
        ws = torch.empty(hip.bn_workspace_bytes(n, h, w, co, nseg), dtype=torch.uint8, device=dev)
        hip.bn_train_stats(hip.nhwc(y0), nseg, gamma, beta, 1e-5, 0.1, False, None, None, smean, sinv, scale, shift, ws)
        ga_ref = torch.empty(n, h, w, co, device=dev)
        hip.conv_igemm(hip.nhwc(dy1), h, w, 1, hip.TAPS_3X3, wb, co, None, hip.nhwc(ga_ref))
        ga = torch.empty(n, h, w, co, device=dev)
        ntiles, tpx = hip.igemm_bn_bwd_tiles(hip.nhwc(dy1), h, w, 1, hip.TAPS_3X3, wb, co, hip.nhwc(ga))
        assert ntiles > 0 and ntiles * tpx == n * h * w
        rec = torch.empty(co * ntiles * 2, device=dev)
        hip.conv_igemm(hip.nhwc(dy1), h, w, 1, hip.TAPS_3X3, wb, co, None, hip.nhwc(ga),
                       bn_bwd=(y0, nseg, smean, sinv, scale, shift, rec))
        assert torch.equal(ga, ga_ref)  # the epilogue sums do not touch the stored output
        outs = []
        for fused in (False, True):
            o = [torch.empty(n, h, w, co, device=dev)] + [torch.empty(co, device=dev) for _ in range(3)]
            if fused:
                hip.bn_relu_backward_tiles(hip.nhwc(y0), hip.nhwc(ga), nseg, smean, sinv, gamma, scale, shift, rec,
                                           ntiles, o[1], o[2], o[3], hip.nhwc(o[0]), ws)
            else:
                hip.bn_relu_backward(hip.nhwc(y0), hip.nhwc(ga_ref), nseg, smean, sinv, gamma, scale, shift, o[1], o[2],
                                     o[3], hip.nhwc(o[0]), ws)
            outs.append(o)
        for a, b in zip(outs[0][:3], outs[1][:3]):  # dy, dgamma, dbeta
            assert rel(a, b) < 2e-6
        # conv-bias grad sum(dy): exactly 0 in real arithmetic (BatchNorm removes the mean), rounding noise here
        scale_dy = outs[0][0].abs().max().item()
        assert outs[0][3].abs().max().item() < 1e-3 * scale_dy and outs[1][3].abs().max().item() < 1e-3 * scale_dy
    finally:
        hip.set_conv_math(prev_m)


@pytest.mark.parametrize('n,h,w,ci,co', [(2, 4, 32, 64, 64), (3, 6, 16, 128, 192), (1, 32, 64, 64, 128),
                                         (2, 16, 16, 512, 512)])
def test_wgrad_halo(dev, n, h, w, ci, co):
    """The halo weight grad (16x16x32 MFMA, x3) against torch fp32, incl. split-K slabs."""
    from multimodal_siamese_cd_amd import hip
    prev_m = hip.set_conv_math('x3')
    try:
        g = torch.Generator().manual_seed(5 + ci + co + h)
        x = torch.randn(n, h, w, ci, generator=g)
        dy = torch.randn(n, h, w, co, generator=g)
        wt = torch.empty(co, ci, 3, 3)
        ref_dw = torch.nn.grad.conv2d_weight(nchw(x), wt.shape, nchw(dy), padding=1)
        d, nsplit, nbytes = hip.wgrad_plan(hip.nhwc(dy.to(dev)), hip.nhwc(x.to(dev)), 1, hip.TAPS_3X3)
        slabs = torch.empty(nbytes // 4, device=dev)
        hip.conv_wgrad(d, slabs)
        dw = torch.empty(co, ci, 3, 3, device=dev)
        hip.wgrad_finalize(slabs, nsplit, co, 9, ci, 0, ci, dw)
        assert rel(dw, ref_dw) < TOL
    finally:
        hip.set_conv_math(prev_m)


@pytest.mark.parametrize('n,h,w,co', [(2, 8, 64, 64), (1, 4, 64, 128), (3, 2, 64, 72), (2, 24, 48, 64)])
def test_conv_16_channel_source_forward(dev, n, h, w, co):
    """The input layer's forward conv (16-channel source, two taps per 32-deep MFMA step) against fp64 under
    x3 / x5 / bf16 / h2 (with the input's bound; without one h2 keeps x3), with bias and fused BatchNorm tile
    statistics (against the host on the kernel's output)."""
    from multimodal_siamese_cd_amd import hip
    ci = 16
    g = torch.Generator().manual_seed(n * w + co)
    spread = lambda *s: (torch.randn(*s, generator=g, dtype=torch.float64)
                         * 10 ** (4 * torch.rand(*s, generator=g, dtype=torch.float64) - 2)).float()
    x = spread(n, h, w, ci)
    wt = (torch.randn(co, ci, 3, 3, generator=g, dtype=torch.float64) / (3 * ci ** 0.5)).float()
    b = torch.randn(co, generator=g)
    ref = nhwc_t(F.conv2d(nchw(x).double(), wt.double(), b.double(), padding=1))
    errs = {}
    for m in ('f32', 'x3', 'x5', 'bf16', 'h2'):
        prev = hip.set_conv_math(m)
        try:
            xd, wd, bd = x.to(dev), wt.to(dev), b.to(dev)
            wpk = hip.pack_conv3x3(wd, 0)
            y = torch.empty(n, h, w, co, device=dev)
            xb = None
            if m == 'h2':
                xb = torch.zeros(1, device=dev)
                hip.absmax_bound(hip.nhwc(xd), xb)
                assert hip.igemm_arith(hip.nhwc(xd), h, w, 1, hip.TAPS_3X3, wpk, co, hip.nhwc(y)) == 'x3'
            if m == 'f32':
                hip.conv_igemm(hip.nhwc(xd), h, w, 1, hip.TAPS_3X3, wpk, co, bd, hip.nhwc(y))
            else:
                assert hip.igemm_arith(hip.nhwc(xd), h, w, 1, hip.TAPS_3X3, wpk, co, hip.nhwc(y), src_bound=xb) == m
                ntiles, tpx = hip.igemm_stat_tiles(hip.nhwc(xd), h, w, 1, hip.TAPS_3X3, wpk, co, hip.nhwc(y),
                                                   src_bound=xb)
                assert tpx == 128 and ntiles * tpx == n * h * w
                rec = torch.empty(ntiles * co * 2, device=dev)
                hip.conv_igemm(hip.nhwc(xd), h, w, 1, hip.TAPS_3X3, wpk, co, bd, hip.nhwc(y), stat_rec=rec,
                               src_bound=xb)
                tw = next(c for c in (16, 32, 64) if w % c == 0 and h % (128 // c) == 0)
                tr = 128 // tw
                yy = y.double().cpu().reshape(n, h // tr, tr, w // tw, tw, co).permute(0, 1, 3, 2, 4, 5)
                yy = yy.reshape(-1, 128, co)
                r = rec.double().cpu().reshape(ntiles, co, 2)
                assert rel(r[..., 0], yy.mean(1)) < 2e-6
                assert rel(r[..., 1], ((yy - yy.mean(1, keepdim=True)) ** 2).sum(1)) < 2e-5
        finally:
            hip.set_conv_math(prev)
        errs[m] = rel(y, ref)
    assert errs['x3'] <= 2 * errs['f32'] + 1e-7 and errs['x5'] < 1e-5 and errs['bf16'] < 2e-2, errs
    assert errs['h2'] <= 2 * errs['f32'] + 1e-7, errs
    # without a bound the h2-split weights are ignored and the per-tap x3 kernel runs: the same accuracy
    prev = hip.set_conv_math('h2')
    try:
        y2 = torch.empty(n, h, w, co, device=dev)
        hip.conv_igemm(hip.nhwc(x.to(dev)), h, w, 1, hip.TAPS_3X3, hip.pack_conv3x3(wt.to(dev), 0), co, b.to(dev),
                       hip.nhwc(y2))
    finally:
        hip.set_conv_math(prev)
    assert rel(y2, ref) <= 2 * errs['f32'] + 1e-7


@pytest.mark.parametrize('n,h,w,co', [(2, 4, 32, 64), (3, 32, 48, 128), (1, 2, 16, 64)])
def test_wgrad_16_channel_source(dev, n, h, w, co):
    """The input layer's weight grad (5 bands padded to 16 channels) on its own halo kernel: against fp64 under
    x3 / x5 / bf16 (the arithmetic query names the kernel's planes), and reading the source through BN-apply +
    ReLU bit-identical to the materialised activation."""
    from multimodal_siamese_cd_amd import hip
    ci = 16
    g = torch.Generator().manual_seed(n * h + co)
    spread = lambda *s: (torch.randn(*s, generator=g, dtype=torch.float64)
                         * 10 ** (4 * torch.rand(*s, generator=g, dtype=torch.float64) - 2)).float()
    x, dy = spread(n, h, w, ci), spread(n, h, w, co)
    ref = torch.nn.grad.conv2d_weight(nchw(x).double(), (co, ci, 3, 3), nchw(dy).double(), padding=1)

    def wgrad(src, dyd, sbn=None):
        d, nsplit, nbytes = hip.wgrad_plan(hip.nhwc(dyd), hip.nhwc(src), 1, hip.TAPS_3X3, sbn)
        slabs = torch.empty(nbytes // 4, device=dev)
        hip.conv_wgrad(d, slabs)
        dw = torch.empty(co, ci, 3, 3, device=dev)
        hip.wgrad_finalize(slabs, nsplit, co, 9, ci, 0, ci, dw)
        return d, dw

    errs = {}
    for m in ('f32', 'x3', 'x5', 'bf16'):
        prev = hip.set_conv_math(m)
        try:
            d, dw = wgrad(x.to(dev), dy.to(dev))
            if m != 'f32':
                assert hip.wgrad_arith(d) == m
        finally:
            hip.set_conv_math(prev)
        errs[m] = rel(dw, ref)
    assert errs['x3'] <= 2 * errs['f32'] + 1e-7 and errs['x5'] < 1e-5 and errs['bf16'] < 2e-2, errs
    prev = hip.set_conv_math('x3')
    try:
        y = torch.randn(2 * n, h, w, ci, generator=g).to(dev)
        dy2 = torch.randn(2 * n, h, w, co, generator=g).to(dev)
        sc = (torch.rand(2 * ci, generator=g) * 2 - 0.5).to(dev)
        sh = torch.randn(2 * ci, generator=g).to(dev)
        a = torch.empty_like(y)
        hip.bn_relu_apply(hip.nhwc(y), 2, sc, sh, hip.nhwc(a))
        assert hip.wgrad_src_bn_supported(hip.nhwc(dy2), hip.nhwc(y), 1, hip.TAPS_3X3, (sc, sh, 2))
        assert torch.equal(wgrad(a, dy2)[1], wgrad(y, dy2, (sc, sh, 2))[1])
    finally:
        hip.set_conv_math(prev)


@pytest.mark.parametrize('n,h,w,c,nseg', [(4, 16, 16, 8, 2), (2, 33, 17, 64, 2), (2, 64, 64, 16, 1), (6, 8, 8, 512, 2)])
def test_batchnorm_relu_train_forward_backward(dev, n, h, w, c, nseg):
    from multimodal_siamese_cd_amd import hip
    g = torch.Generator().manual_seed(n * h + c)
    y = (torch.randn(n, h, w, c, generator=g) * 3 + 5).requires_grad_(True)  # mean >> std stresses the variance
    gamma = (1 + 0.1 * torch.randn(c, generator=g)).requires_grad_(True)
    beta = (0.1 * torch.randn(c, generator=g)).requires_grad_(True)
    rm0, rv0 = torch.randn(c, generator=g), torch.rand(c, generator=g) + 0.5
    rm, rv = rm0.clone(), rv0.clone()
    outs = []
    per = n // nseg
    for s in range(nseg):
        ys = nchw(y[s * per:(s + 1) * per])
        outs.append(nhwc_t(F.relu(F.batch_norm(ys, rm, rv, gamma, beta, True, 0.1, 1e-5))))
    ref = torch.cat(outs)
    ga = torch.randn(n, h, w, c, generator=g)
    ref.backward(ga)

    yd = y.detach().to(dev)
    smean, sinv, scale, shift = (torch.empty(nseg * c, device=dev) for _ in range(4))
    rmd, rvd = rm0.to(dev), rv0.to(dev)
    ws = torch.empty(hip.bn_workspace_bytes(n, h, w, c, nseg), dtype=torch.uint8, device=dev)
    gd, bd = gamma.detach().to(dev), beta.detach().to(dev)
    hip.bn_train_stats(hip.nhwc(yd), nseg, gd, bd, 1e-5, 0.1, True, rmd, rvd, smean, sinv, scale, shift, ws)
    a = torch.empty_like(yd)
    hip.bn_relu_apply(hip.nhwc(yd), nseg, scale, shift, hip.nhwc(a))
    assert rel(a, ref) < 1e-5
    assert rel(rmd, rm) < 1e-6 and rel(rvd, rv) < 1e-6
    dy = torch.empty_like(yd)
    dgam, dbet, dbias = (torch.empty(c, device=dev) for _ in range(3))
    hip.bn_relu_backward(hip.nhwc(yd), hip.nhwc(ga.to(dev)), nseg, smean, sinv, gd, scale, shift, dgam, dbet, dbias,
                         hip.nhwc(dy), ws)
    assert rel(dy, y.grad) < 1e-4
    assert rel(dgam, gamma.grad) < 1e-5 and rel(dbet, beta.grad) < 1e-5
    assert (dbias.cpu() - y.grad.sum((0, 1, 2))).abs().max() < 1e-3 * y.grad.abs().max()


@pytest.mark.parametrize('math', ['x3', 'bf16', 'h2'])
@pytest.mark.parametrize('n,h,w,co,nseg,tiles', [(4, 8, 32, 64, 2, False), (2, 4, 16, 128, 1, False),
                                                 (4, 16, 16, 64, 2, True)])
def test_wgrad_c16_deferred_bn_backward(dev, math, n, h, w, co, nseg, tiles):
    """The input layer's weight grad forming dy = BN-backward(y, da) while staging (scd_wgrad_t.rows_y, coefficients
    from scd_bn_relu_backward_coef) equals the BatchNorm backward's materialised dy fed to the same kernel, bit for
    bit; dgamma / dbeta are the full backward's; the conv-bias grad (sum dy, 0 in exact arithmetic) stays ~0.
    h2: the coefficient pass's dy bound (from the statistics and a bound of da) bounds the materialised dy, both
    weight grads run h2 under that bound, and the result is within 2e-6 of the fp64 weight grad."""
    from multimodal_siamese_cd_amd import hip
    ci = 16
    g = torch.Generator().manual_seed(n * co + nseg + h)
    y = (torch.randn(n, h, w, co, generator=g) * 2 + 0.3).to(dev)
    da = torch.randn(n, h, w, co, generator=g).to(dev)
    x = torch.randn(n, h, w, ci, generator=g).to(dev)
    gamma = (torch.rand(co, generator=g) + 0.5).to(dev)
    beta = torch.randn(co, generator=g).to(dev)
    smean, sinv, scale, shift = (torch.empty(nseg * co, device=dev) for _ in range(4))
    ws = torch.empty(hip.bn_workspace_bytes(n, h, w, co, nseg), dtype=torch.uint8, device=dev)
    hip.bn_train_stats(hip.nhwc(y), nseg, gamma, beta, 1e-5, 0.1, False, None, None, smean, sinv, scale, shift, ws)
    rec, ntiles = None, 0
    if tiles:  # partial sums as a conv epilogue would record them: one tile per 128 pixels, from the host
        per, tp = n // nseg, 128
        yy = y.double().cpu().reshape(-1, tp, co)
        z = torch.where(y.double().cpu() * scale.double().cpu().reshape(nseg, 1, 1, 1, co).repeat_interleave(
            per, 0).reshape(n, 1, 1, co) + shift.double().cpu().reshape(nseg, co).repeat_interleave(per, 0).reshape(
            n, 1, 1, co) > 0, da.double().cpu(), torch.zeros(()).double())
        mu = smean.double().cpu().reshape(nseg, co).repeat_interleave(per, 0).reshape(n, 1, 1, co)
        iv = sinv.double().cpu().reshape(nseg, co).repeat_interleave(per, 0).reshape(n, 1, 1, co)
        xh = ((y.double().cpu() - mu) * iv).reshape(-1, tp, co)
        zz = z.reshape(-1, tp, co)
        ntiles = zz.shape[0]
        rec = torch.stack([zz.sum(1), (zz * xh).sum(1)], -1).permute(1, 0, 2).contiguous().float().to(dev)
    prev = hip.set_conv_math(math)
    try:
        dy = torch.empty_like(y)
        o = [torch.empty(co, device=dev) for _ in range(3)]
        if tiles:
            hip.bn_relu_backward_tiles(hip.nhwc(y), hip.nhwc(da), nseg, smean, sinv, gamma, scale, shift, rec, ntiles,
                                       *o, hip.nhwc(dy), ws)
        else:
            hip.bn_relu_backward(hip.nhwc(y), hip.nhwc(da), nseg, smean, sinv, gamma, scale, shift, *o, hip.nhwc(dy), ws)
        assert hip.wgrad_rows_bn_supported(hip.nhwc(da), hip.nhwc(x), 1, hip.TAPS_3X3)

        coef = torch.empty(nseg * co * 2, device=dev)
        q = [torch.empty(co, device=dev) for _ in range(3)]
        da_bound = da.abs().max().reshape(1) if math == 'h2' else None
        dy_bound = torch.zeros(1, device=dev) if math == 'h2' else None
        x_bound = x.abs().max().reshape(1) if math == 'h2' else None
        hip.bn_relu_backward_coef(hip.nhwc(y), hip.nhwc(da), nseg, smean, sinv, gamma, scale, shift, rec, ntiles, coef,
                                  *q, ws, da_bound, dy_bound)

        def wgrad(rows, rows_bn=None):
            d, nsplit, nbytes = hip.wgrad_plan(hip.nhwc(rows), hip.nhwc(x), 1, hip.TAPS_3X3, None, dy_bound, x_bound,
                                               rows_bn=rows_bn)
            assert hip.wgrad_arith(d) == math
            slabs = torch.empty(nbytes // 4, device=dev)
            hip.conv_wgrad(d, slabs)
            dw = torch.empty(co, ci, 3, 3, device=dev)
            hip.wgrad_finalize(slabs, nsplit, co, 9, ci, 0, ci, dw)
            return dw

        ref = wgrad(dy)
        out = wgrad(da, (hip.nhwc(y), nseg, smean, sinv, gamma, scale, shift, coef))
    finally:
        hip.set_conv_math(prev)
    assert torch.equal(out, ref)
    if math == 'h2':
        amax = dy.abs().max().item()
        assert amax <= dy_bound.item() < 4096 * amax * (n * h * w) ** 0.5
        exact = torch.nn.grad.conv2d_weight(x.double().cpu().permute(0, 3, 1, 2), (co, ci, 3, 3),
                                            dy.double().cpu().permute(0, 3, 1, 2), padding=1)
        assert rel(out.double().cpu(), exact) < 2e-6
    assert torch.equal(q[0], o[0]) and torch.equal(q[1], o[1])
    scale_dy = dy.abs().max().item()
    assert q[2].abs().max().item() < 1e-3 * scale_dy and o[2].abs().max().item() < 1e-3 * scale_dy


@pytest.mark.parametrize('math,dt,co,ci,nseg,src_bn', [
    ('h2', torch.float32, 128, 64, 2, False), ('h2', torch.float32, 256, 128, 1, True),
    ('bf16', torch.bfloat16, 64, 64, 2, False), ('bf16', torch.bfloat16, 128, 64, 1, True),
    ('bf16', torch.bfloat16, 256, 128, 2, True), ('bf16', torch.bfloat16, 64, 128, 1, True),
    ('bf16', torch.float32, 64, 128, 2, False)])
def test_halo_wgrad_forms_and_stores_dy(dev, math, dt, co, ci, nseg, src_bn):
    """ABI 8: the 64-channel-multiple halo weight grad with the rows' BatchNorm backward (scd_wgrad_t.rows_y) stores
    the dY it forms (rows_out) bit for bit as scd_bn_relu_backward writes it, raises rows_out_bound to exactly max |dY|,
    and its weight grad equals the weight grad of the materialised dY under the same operand bounds, bit for bit.  The
    blocks of channel tile 0 store: ci = 128 has two channel tiles, so each dY element is still written once."""
    from multimodal_siamese_cd_amd import hip
    n, h, w = 4, 32, 32
    g = torch.Generator().manual_seed(co + ci + nseg)
    y = (torch.randn(n, h, w, co, generator=g) * 2 + 0.3).to(dev).to(dt)
    da = torch.randn(n, h, w, co, generator=g).to(dev).to(dt)
    x = torch.randn(n, h, w, ci, generator=g).to(dev).to(dt)
    gamma = (torch.rand(co, generator=g) + 0.5).to(dev)
    beta = torch.randn(co, generator=g).to(dev)
    smean, sinv, scale, shift = (torch.empty(nseg * co, device=dev) for _ in range(4))
    ws = torch.empty(hip.bn_workspace_bytes(n, h, w, co, nseg), dtype=torch.uint8, device=dev)
    hip.bn_train_stats(hip.nhwc(y), nseg, gamma, beta, 1e-5, 0.1, False, None, None, smean, sinv, scale, shift, ws)
    xbn = None
    if src_bn:  # the weight grad's source read through its own BatchNorm + ReLU (the decoder's second conv)
        xbn = ((torch.rand(2 * ci, generator=g) + 0.5).to(dev), torch.randn(2 * ci, generator=g).to(dev), 2)
    prev = hip.set_conv_math(math)
    try:
        dy = torch.empty_like(y)
        o = [torch.empty(co, device=dev) for _ in range(3)]
        hip.bn_relu_backward(hip.nhwc(y), hip.nhwc(da), nseg, smean, sinv, gamma, scale, shift, *o, hip.nhwc(dy), ws)
        h2 = math == 'h2'
        da_bound = da.float().abs().max().reshape(1) if h2 else None
        dy_bound = torch.zeros(1, device=dev) if h2 else None
        if h2:
            xa = x.float()
            if src_bn:
                sc2, sh2 = xbn[0].reshape(2, 1, 1, 1, ci), xbn[1].reshape(2, 1, 1, 1, ci)
                xa = torch.relu(xa.reshape(2, n // 2, h, w, ci) * sc2 + sh2)
            x_bound = xa.abs().max().reshape(1)
        else:
            x_bound = None
        assert hip.wgrad_rows_bn_supported(hip.nhwc(da), hip.nhwc(x), 1, hip.TAPS_3X3, xbn, dy_bound, x_bound)
        coef = torch.empty(nseg * co * 2, device=dev)
        q = [torch.empty(co, device=dev) for _ in range(3)]
        hip.bn_relu_backward_coef(hip.nhwc(y), hip.nhwc(da), nseg, smean, sinv, gamma, scale, shift, None, 0, coef,
                                  *q, ws, da_bound, dy_bound)
        dy_out = torch.full_like(y, float('nan'))
        out_bound = torch.zeros(1, device=dev)

        def wgrad(rows, rows_bn=None, rows_out=None):
            d, nsplit, nbytes = hip.wgrad_plan(hip.nhwc(rows), hip.nhwc(x), 1, hip.TAPS_3X3, xbn, dy_bound, x_bound,
                                               rows_bn=rows_bn, rows_out=rows_out, rows_out_bound=out_bound)
            assert hip.wgrad_arith(d) == math
            slabs = torch.empty(nbytes // 4, device=dev)
            hip.conv_wgrad(d, slabs)
            dw = torch.empty(co, ci, 3, 3, device=dev)
            hip.wgrad_finalize(slabs, nsplit, co, 9, ci, 0, ci, dw)
            return dw

        ref = wgrad(dy)
        out = wgrad(da, (hip.nhwc(y), nseg, smean, sinv, gamma, scale, shift, coef), hip.nhwc(dy_out))
        torch.cuda.synchronize()
    finally:
        hip.set_conv_math(prev)
    assert torch.equal(dy_out, dy)
    assert out_bound.item() == dy.float().abs().max().item()
    assert torch.equal(out, ref)
    if h2:
        assert dy.float().abs().max().item() <= dy_bound.item()


def test_batchnorm_eval(dev):
    from multimodal_siamese_cd_amd import hip
    g = torch.Generator().manual_seed(5)
    n, h, w, c = 2, 8, 8, 32
    y = torch.randn(n, h, w, c, generator=g)
    gamma, beta = torch.randn(c, generator=g), torch.randn(c, generator=g)
    rm, rv = torch.randn(c, generator=g), torch.rand(c, generator=g) + 0.1
    ref = nhwc_t(F.relu(F.batch_norm(nchw(y), rm, rv, gamma, beta, False, 0.1, 1e-5)))
    scale, shift = torch.empty(c, device=dev), torch.empty(c, device=dev)
    hip.bn_eval_coeffs(c, gamma.to(dev), beta.to(dev), rm.to(dev), rv.to(dev), 1e-5, scale, shift)
    a = torch.empty(n, h, w, c, device=dev)
    hip.bn_relu_apply(hip.nhwc(y.to(dev)), 1, scale, shift, hip.nhwc(a))
    assert rel(a, ref) < 1e-5


@pytest.mark.parametrize('n,h,w,c', [(2, 16, 16, 8), (2, 7, 9, 64), (1, 32, 32, 512)])
def test_maxpool_forward_indices_and_feature_grad(dev, n, h, w, c):
    from multimodal_siamese_cd_amd import hip
    g = torch.Generator().manual_seed(h * w + c)
    x = F.relu(torch.randn(n, h, w, c, generator=g))  # ReLU outputs: many ties at 0 (first max wins)
    x[0, 0, 1, 0] = float('nan')
    xc = nchw(x).requires_grad_(True)
    ref, ref_idx = F.max_pool2d(xc, 2, return_indices=True)
    ho, wo = h // 2, w // 2
    xd = x.to(dev)
    y = torch.empty(n, ho, wo, c, device=dev)
    idx = torch.empty(n, ho, wo, c, dtype=torch.uint8, device=dev)
    hip.maxpool2_fwd(hip.nhwc(xd), hip.nhwc(y), idx)
    yc = y.cpu()
    assert torch.equal(torch.isnan(yc), torch.isnan(nhwc_t(ref.detach())))
    assert torch.equal(torch.nan_to_num(yc, 0.0), torch.nan_to_num(nhwc_t(ref.detach()), 0.0))
    # decode aten's flat indices to window positions
    ri = nhwc_t(ref_idx)
    oy = torch.arange(ho).view(1, ho, 1, 1)
    ox = torch.arange(wo).view(1, 1, wo, 1)
    win = ((ri // w) - 2 * oy) * 2 + ((ri % w) - 2 * ox)
    assert torch.equal(idx.cpu().long(), win)
    # backward + Siamese skip add: gx = pool_bwd(gy) + sign * gskip
    gy = torch.randn(n, ho, wo, c, generator=g)
    ref.backward(nchw(gy))
    gskip = torch.randn(n // 2 if n > 1 else 1, h, w, c, generator=g)
    gx = torch.empty(n, h, w, c, device=dev)
    mode = 1 if n % 2 == 0 else 0
    gyd, gsd = gy.to(dev), gskip.to(dev)
    hip.feature_grad(hip.nhwc(gyd), idx, hip.nhwc(gsd), mode, hip.nhwc(gx))
    sgn = torch.ones(n, 1, 1, 1)
    if mode == 1:
        sgn[: n // 2] = -1
    want = nhwc_t(xc.grad) + sgn * gskip.repeat(n // gskip.shape[0], 1, 1, 1)
    assert torch.allclose(gx.cpu(), want, atol=1e-6)


@pytest.mark.parametrize('n,h,w,c,nseg', [(4, 16, 16, 64, 2), (2, 7, 9, 32, 1), (4, 32, 32, 128, 2)])
def test_bn_relu_fused_pool_and_diff(dev, n, h, w, c, nseg):
    """MaxPool2d and the Siamese difference reading y through BN-apply + ReLU == the same ops on the
    materialised activation (bit-identical, argmax bytes included)."""
    from multimodal_siamese_cd_amd import hip
    g = torch.Generator().manual_seed(n * c + h)
    y = torch.randn(n, h, w, c, generator=g).to(dev)
    sc = (torch.rand(nseg * c, generator=g) * 2 - 0.5).to(dev)
    sh = torch.randn(nseg * c, generator=g).to(dev)
    a = torch.empty_like(y)
    hip.bn_relu_apply(hip.nhwc(y), nseg, sc, sh, hip.nhwc(a))
    p_ref, p = (torch.empty(n, h // 2, w // 2, c, device=dev) for _ in range(2))
    i_ref, i = (torch.empty(n, h // 2, w // 2, c, device=dev, dtype=torch.uint8) for _ in range(2))
    hip.maxpool2_fwd(hip.nhwc(a), hip.nhwc(p_ref), i_ref)
    hip.bn_relu_maxpool2_fwd(hip.nhwc(y), nseg, sc, sh, hip.nhwc(p), i)
    assert torch.equal(p, p_ref) and torch.equal(i, i_ref)
    sc2, sh2 = (sc, sh) if nseg == 2 else (torch.cat([sc, sc]), torch.cat([sh, sh]))
    d_ref = torch.empty(n // 2, h, w, c, device=dev)
    hip.siamese_diff(hip.nhwc(a), hip.nhwc(d_ref))
    buf = torch.full((n // 2, h, w, c + 8), 7.0, device=dev)  # write into a concat slice; the rest untouched
    hip.bn_relu_siamese_diff(hip.nhwc(y), sc2, sh2, hip.nhwc(buf, 0, c))
    assert torch.equal(buf[..., :c], d_ref) and bool((buf[..., c:] == 7.0).all())
    if h % 2 == 0 and w % 2 == 0:  # the one-pass difference + pooling of both branches
        p_ref2, i_ref2 = torch.empty_like(p), torch.empty_like(i)
        hip.bn_relu_maxpool2_fwd(hip.nhwc(y), 2, sc2, sh2, hip.nhwc(p_ref2), i_ref2)
        p2, i2 = torch.full_like(p, 3.0), torch.zeros_like(i)
        buf2 = torch.full((n // 2, h, w, c + 8), 7.0, device=dev)
        hip.bn_relu_pool_diff(hip.nhwc(y), sc2, sh2, hip.nhwc(buf2, 0, c), hip.nhwc(p2), i2)
        assert torch.equal(buf2, buf) and torch.equal(p2, p_ref2) and torch.equal(i2, i_ref2)


@pytest.mark.parametrize('n,h,w,c,mode,parts', [(4, 16, 16, 64, 1, 'both'), (4, 9, 7, 32, 1, 'both'),
                                                 (2, 8, 8, 128, 1, 'skip'), (4, 10, 12, 64, 0, 'both'),
                                                 (2, 16, 8, 64, 0, 'pool')])
def test_bn_relu_backward_pooled(dev, n, h, w, c, mode, parts):
    """The BatchNorm + ReLU backward forming its incoming gradient on the fly (maxpool_bwd -/+ skip) over 2x2 cells:
    feature_grad followed by bn_relu_backward (dy, dgamma, dbeta, conv-bias grad) up to the order of the per-chunk
    sums (2e-6).  (The per-pixel walk, -DSCD_BN_POOLED_CELLS=0, is bit-identical to the unfused pair.)"""
    from multimodal_siamese_cd_amd import hip
    g = torch.Generator().manual_seed(n * h * w + c + mode)
    nseg = 2
    y = (torch.randn(n, h, w, c, generator=g) * 2 + 0.3).to(dev)
    gamma = (torch.rand(c, generator=g) + 0.5).to(dev)
    beta = torch.randn(c, generator=g).to(dev)
    smean, sinv, scale, shift = (torch.empty(nseg * c, device=dev) for _ in range(4))
    ws = torch.empty(hip.bn_workspace_bytes(n, h, w, c, nseg), dtype=torch.uint8, device=dev)
    hip.bn_train_stats(hip.nhwc(y), nseg, gamma, beta, 1e-5, 0.1, False, None, None, smean, sinv, scale, shift, ws)
    gy = idx = gs = None
    if parts in ('both', 'pool'):
        x = torch.randn(n, h, w, c, generator=g).to(dev)
        gy = torch.randn(n, h // 2, w // 2, c, generator=g).to(dev)
        idx = torch.empty(n, h // 2, w // 2, c, dtype=torch.uint8, device=dev)
        hip.maxpool2_fwd(hip.nhwc(x), hip.nhwc(torch.empty_like(gy)), idx)
    if parts in ('both', 'skip'):
        gs = torch.randn(n // 2 if mode == 1 else n, h, w, c + 8, generator=g).to(dev)[..., 4:4 + c]  # strided view
    nh = lambda t: hip.nhwc(t) if t is not None else hip._NULL
    ga = torch.empty_like(y)
    hip.feature_grad(nh(gy), idx, nh(gs), mode, hip.nhwc(ga))
    outs = []
    for pooled in (False, True):
        dy = torch.empty_like(y)
        dg, db, dbias = (torch.empty(c, device=dev) for _ in range(3))
        if pooled:
            hip.bn_relu_backward_pooled(hip.nhwc(y), nh(gy), idx, nh(gs), mode, nseg, smean, sinv, gamma, scale,
                                        shift, dg, db, dbias, hip.nhwc(dy), ws)
        else:
            hip.bn_relu_backward(hip.nhwc(y), hip.nhwc(ga), nseg, smean, sinv, gamma, scale, shift, dg, db, dbias,
                                 hip.nhwc(dy), ws)
        outs.append((dy, dg, db, dbias))
    for a, b in zip(outs[0][:3], outs[1][:3]):
        assert rel(a, b) < 2e-6
    # the conv-bias grad is a sum of dy that cancels to ~0 (a pre-BN bias): judged against the sum of |dy|
    assert ((outs[0][3] - outs[1][3]).abs() <= 2e-6 * outs[0][0].abs().sum(dim=(0, 1, 2))).all()


def test_siamese_diff(dev):
    from multimodal_siamese_cd_amd import hip
    a = torch.randn(6, 5, 7, 16)
    d = torch.empty(3, 5, 7, 16, device=dev)
    hip.siamese_diff(hip.nhwc(a.to(dev)), hip.nhwc(d))
    assert torch.equal(d.cpu(), a[3:] - a[:3])


@pytest.mark.parametrize('n,nseg,c,n_out,h,w', [(4, 2, 64, 1, 16, 24), (6, 3, 32, 2, 7, 9), (2, 1, 128, 1, 5, 13),
                                                 (6, 2, 16, 4, 11, 3)])
def test_head_conv1x1_fused_bn_segments(dev, n, nseg, c, n_out, h, w):
    """The head read through its BatchNorm + ReLU (scd_conv1x1_fwd_bn): each of the nseg image segments takes its own
    coefficients (the segment of a pixel is found with a multiply-shift, not an int64 division)."""
    from multimodal_siamese_cd_amd import hip
    g = torch.Generator().manual_seed(n * c + nseg)
    y = torch.randn(n, h, w, c, generator=g)
    sc = torch.rand(nseg, c, generator=g) + 0.5
    sh = torch.randn(nseg, c, generator=g) * 0.2
    wt = torch.randn(n_out, c, generator=g)
    b = torch.randn(n_out, generator=g)
    seg = torch.arange(n) // (n // nseg)
    a = torch.relu(y.double() * sc.double()[seg][:, None, None, :] + sh.double()[seg][:, None, None, :])
    ref = torch.einsum('nhwc,oc->nohw', a, wt.double()) + b.double()[None, :, None, None]
    o = torch.empty(n, n_out, h, w, device=dev)
    hip.conv1x1_fwd_bn(hip.nhwc(y.to(dev)), sc.reshape(-1).to(dev), sh.reshape(-1).to(dev), nseg, wt.to(dev),
                       b.to(dev), n_out, o)
    assert rel(o, ref) < TOL


@pytest.mark.parametrize('c,n_out,h,w', [(64, 1, 16, 24), (8, 1, 16, 24), (128, 1, 16, 24), (16, 3, 16, 24),
                                         (64, 1, 7, 9), (32, 4, 5, 13)])  # odd sizes: ragged last pixel group
def test_head_conv1x1(dev, c, n_out, h, w):
    from multimodal_siamese_cd_amd import hip
    g = torch.Generator().manual_seed(c + n_out)
    n = 2
    x = torch.randn(n, c, h, w, generator=g, requires_grad=True)
    wt = torch.randn(n_out, c, 1, 1, generator=g, requires_grad=True)
    b = torch.randn(n_out, generator=g, requires_grad=True)
    out = F.conv2d(x, wt, b)
    gout = torch.randn(out.shape, generator=g)
    out.backward(gout)
    xd = nhwc_t(x.detach()).to(dev)
    o = torch.empty(n, n_out, h, w, device=dev)
    wd = wt.detach().reshape(n_out, c).contiguous().to(dev)
    hip.conv1x1_fwd(hip.nhwc(xd), wd, b.detach().to(dev), n_out, o)
    assert rel(o, out) < TOL
    gx = torch.empty_like(xd)
    gw = torch.empty(n_out, c, 1, 1, device=dev)
    gb = torch.empty(n_out, device=dev)
    ws = torch.empty(hip.conv1x1_workspace_bytes(hip.nhwc(xd), n_out), dtype=torch.uint8, device=dev)
    hip.conv1x1_bwd(hip.nhwc(xd), wd, gout.to(dev), n_out, hip.nhwc(gx), False, gw, gb, ws)
    assert rel(gx, nhwc_t(x.grad)) < TOL
    assert rel(gw, wt.grad) < TOL and rel(gb, b.grad) < TOL


@pytest.mark.parametrize('n,soft', [(2 * 64 * 64, False), (3 * 97 * 31, False), (2 * 32 * 32, True)])
def test_power_jaccard(dev, n, soft):
    from multimodal_siamese_cd_amd import engine
    g = torch.Generator().manual_seed(n)
    logits = (torch.randn(n, generator=g) * 3).requires_grad_(True)
    if soft:
        t = torch.sigmoid(torch.randn(n, generator=g)).requires_grad_(True)
    else:
        t = (torch.rand(n, generator=g) > 0.9).float()
    ref = O.power_jaccard_loss(logits, t)
    ref.backward()
    ld = logits.detach().to(dev).requires_grad_(True)
    td = t.detach().to(dev).requires_grad_(soft)
    loss = engine.power_jaccard(ld, td)
    loss.backward()
    assert abs(loss.item() - ref.item()) < 1e-6
    assert rel(ld.grad, logits.grad) < 1e-5
    if soft:
        assert rel(td.grad, t.grad) < 1e-5


def test_errors_are_reported(dev):
    from multimodal_siamese_cd_amd import hip
    x = torch.zeros(1, 4, 4, 6, device=dev)  # c=6 not a multiple of 4
    y = torch.zeros(1, 4, 4, 8, device=dev)
    with pytest.raises(RuntimeError, match='multiples of 4'):
        hip.conv_igemm(hip.nhwc(x), 4, 4, 1, hip.TAPS_3X3, torch.zeros(8 * 9 * 6, device=dev), 8, None, hip.nhwc(y))


def test_pack_conv3x3_multi_matches_single_packs(dev):
    """One batched launch == scd_pack_conv3x3 + scd_split_bf16x3_frag per weight, bit for bit (both modes,
    a channel-padded input layer, more jobs than one launch holds)."""
    from multimodal_siamese_cd_amd import hip
    prev = hip.set_conv_math('x3')
    try:
        g = torch.Generator().manual_seed(4)
        shapes = [(64, 10, 16), (64, 64, 64), (128, 64, 64), (24, 200, 200), (512, 512, 512)] * 11
        jobs = []
        for i, (co, ci, cp) in enumerate(shapes):
            w = torch.randn(co, ci, 3, 3, generator=g).to(dev)
            jobs.append((w, i % 2 if ci % 8 == 0 else 0, cp))
        outs = hip.pack_conv3x3_multi(jobs)
        for (w, mode, cp), o in zip(jobs, outs):
            ref = hip.pack_conv3x3(w, mode, ci_pad=cp if mode == 0 else None)
            assert torch.equal(o, ref)
            assert hasattr(o, '_x3') == hasattr(ref, '_x3')
            if hasattr(ref, '_x3'):
                assert torch.equal(o._x3, ref._x3)
    finally:
        hip.set_conv_math(prev)


def test_weight_pack_cache_follows_parameter_updates(dev):
    """engine.packed_conv3x3 packs a model's whole weight group once per forward pass, and repacks after an
    optimizer step, including torch's fused AdamW, which does not bump parameter version counters."""
    from multimodal_siamese_cd_amd import engine, hip
    from multimodal_siamese_cd_amd.utils import experiment_manager as em, networks
    cfg = em.load_cfg('debug')
    net = networks.create_network(cfg).to(dev)
    convs = [m for m in net.modules() if isinstance(m, torch.nn.Conv2d) and m.kernel_size == (3, 3)]
    w = convs[3].weight
    x = torch.rand(1, 5, 64, 64, device=dev)
    with torch.no_grad():
        net(x, x)
    a = engine.packed_conv3x3(w, 0)
    assert engine.packed_conv3x3(w, 0) is a  # cached within the pass
    grp = engine._GROUPS.get(w)
    assert engine._cached(convs[5].weight, engine._pack_key(0, convs[5].in_channels), grp) is not None  # group
    assert torch.equal(a, hip.pack_conv3x3(w.detach(), 0))
    for fused in (False, True):
        opt = torch.optim.AdamW(net.parameters(), lr=1e-2, fused=fused)
        for p in net.parameters():
            p.grad = torch.ones_like(p)
        opt.step()
        with torch.no_grad():
            net(x, x)  # the next forward pass starts a new generation
        b = engine.packed_conv3x3(w, 0)
        assert b is not a and torch.equal(b, hip.pack_conv3x3(w.detach(), 0)), fused
        a = b


@pytest.mark.parametrize('labeled', [[1, 0, 1, 0], [1, 1, 1, 1], [0, 0, 0, 0], [0, 1, 0, 0]])
@pytest.mark.parametrize('kind', ['mmcr', 'dualtask'])
def test_fused_multi_jaccard_matches_oracle(dev, labeled, kind):
    """The fused multi-term Jaccard of the MMCR / dual-task trainers == the oracle's per-term recipe with boolean
    subsets (train_semisupervised.py:78-113, train_supervised_dualtask.py:73-85), incl. all / no labelled samples:
    loss 1e-6 absolute, every gradient 1e-5 relative (the soft target's included)."""
    from multimodal_siamese_cd_amd import trainers
    from multimodal_siamese_cd_amd.utils import experiment_manager as em
    from oracle import siamese_oracle as O
    g = torch.Generator().manual_seed(sum(labeled) + len(kind))
    B, H, W = 4, 24, 20
    outs = [torch.randn(B, 1, H, W, generator=g) * 2 for _ in range(3)]
    batch = {'y_change': (torch.rand(B, 1, H, W, generator=g) > 0.7).float(),
             'y_sem_t1': (torch.rand(B, 1, H, W, generator=g) > 0.5).float(),
             'y_sem_t2': (torch.rand(B, 1, H, W, generator=g) > 0.5).float(),
             'is_labeled': torch.tensor(labeled, dtype=torch.bool)}
    mtype = 'whatevernet' if kind == 'mmcr' else 'dtsiameseunet'
    ref_in = [o.clone().requires_grad_(True) for o in outs]
    ref = O.step_loss(mtype, tuple(ref_in), batch, 0.5)
    ref.backward()
    cfg = em.load_cfg('siamese_mmcr_alpha0500' if kind == 'mmcr' else 'dtsiamese')
    cfg.CONSISTENCY_TRAINER.LOSS_FACTOR = 0.5
    hip_in = [o.to(dev).requires_grad_(True) for o in outs]
    bd = {k: v.to(dev) for k, v in batch.items()}
    loss = trainers.step_loss(cfg, tuple(hip_in), bd)
    loss.backward()
    assert abs(loss.item() - ref.item()) < 1e-6
    for a, b in zip(hip_in, ref_in):
        assert rel(a.grad, b.grad if b.grad is not None else torch.zeros_like(b)) < 1e-5 or (
            b.grad is None and a.grad.abs().max().item() == 0)


@pytest.mark.parametrize('ci,co', [(64, 128), (256, 256), (128, 64), (512, 512)])
def test_halo_math_accuracy_vs_fp64(dev, ci, co):
    """The halo kernels (forward, data grad, weight grad) under f32 / x3 / x5 against fp64 on wide-dynamic-range
    data.  x3 drops products of <= 2^-24 relative size and stays within 2x of the fp32-MFMA error (measured: at
    or below it).  x5 also drops one <= 2^-18 product: measured 2.5e-6..3.9e-6 relative, 1.2-9x the fp32-MFMA
    error (the weight grad's split-K fp32 sums are the most accurate, so its ratio is the largest)."""
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
    for m in ('f32', 'x3', 'x5'):
        prev = hip.set_conv_math(m)
        try:
            xd, dyd, wd = x.to(dev), dy.to(dev), wt.to(dev)
            y = torch.empty(n, h, w, co, device=dev)
            src = hip.nhwc(xd)
            wpk = hip.pack_conv3x3(wd, 0)
            if m != 'f32':
                assert hip.igemm_arith(src, h, w, 1, hip.TAPS_3X3, wpk, co, hip.nhwc(y)) == m
            hip.conv_igemm(src, h, w, 1, hip.TAPS_3X3, wpk, co, None, hip.nhwc(y))
            dx = torch.empty(n, h, w, ci, device=dev)
            hip.conv_igemm(hip.nhwc(dyd), h, w, 1, hip.TAPS_3X3, hip.pack_conv3x3(wd, 1), ci, None, hip.nhwc(dx))
            d, nsplit, nbytes = hip.wgrad_plan(hip.nhwc(dyd), hip.nhwc(xd), 1, hip.TAPS_3X3)
            if m != 'f32':
                assert hip.wgrad_arith(d) == m
            slabs = torch.empty(nbytes // 4, device=dev)
            hip.conv_wgrad(d, slabs)
            dw = torch.empty(co, ci, 3, 3, device=dev)
            hip.wgrad_finalize(slabs, nsplit, co, 9, ci, 0, ci, dw)
        finally:
            hip.set_conv_math(prev)
        errs[m] = (rel(y, ref_y), rel(dx, ref_dx), rel(dw, ref_dw))
    print(errs)
    for k in range(3):  # x3: at most the fp32-MFMA error; x5: below 1e-5 (measured 2.5e-6..3.9e-6)
        assert errs['x3'][k] <= 2 * errs['f32'][k] + 1e-7, ('x3', k, errs)
        assert errs['x5'][k] < 1e-5, ('x5', k, errs)


@pytest.mark.parametrize('n,c,h,w,c_begin,c_count,dst_c,off,ldc', [
    (2, 5, 12, 20, 0, 5, 16, 0, 16),     # Siamese input: 5 bands zero-padded to 16 (float4 path)
    (3, 5, 7, 9, 0, 5, 8, 0, 8),         # fp32-MFMA padding to 8
    (2, 13, 16, 16, 2, 4, 16, 0, 16),    # band subset (dual-stream)
    (2, 5, 11, 13, 0, 5, 5, 5, 16),      # early fusion t2 half: channel offset 5 (scalar path)
    (1, 4, 5, 6, 0, 4, 4, 4, 12),        # aligned channel slice of a wider buffer (float4 path, ldc 12)
    (2, 3, 300, 301, 1, 2, 3, 1, 6),     # more pixels than one grid stride, odd sizes
])
def test_pack_nchw(dev, n, c, h, w, c_begin, c_count, dst_c, off, ldc):
    """scd_pack_nchw vs torch: NCHW band slice -> NHWC channel slice, zero-filled above c_count, and the
    channels outside the slice untouched; the bound output is exactly the max |value| packed (raised, never
    lowered: a larger starting value stays)."""
    from multimodal_siamese_cd_amd import hip
    g = torch.Generator().manual_seed(11)
    x = torch.randn(n, c, h, w, generator=g) * 3
    buf = torch.full((n, h, w, ldc), -7.0, device=dev)
    bound = torch.zeros(1, device=dev)
    hip.pack_nchw(x.to(dev), c_begin, c_count, buf, off, dst_c, bound=bound)
    exp = torch.full((n, h, w, ldc), -7.0)
    exp[..., off:off + dst_c] = 0.0
    exp[..., off:off + c_count] = x[:, c_begin:c_begin + c_count].permute(0, 2, 3, 1)
    assert torch.equal(buf.cpu(), exp)
    assert bound.item() == x[:, c_begin:c_begin + c_count].abs().max().item()
    big = torch.full((1,), 1e6, device=dev)
    hip.pack_nchw(x.to(dev), c_begin, c_count, buf, off, dst_c, bound=big)
    assert big.item() == 1e6


WGRAD_PLANS = [  # n, h, w, ci, co: 64 / 128-row blocks, the 16-channel input-layer kernel, split-K ranges
    (2, 4, 32, 64, 64), (3, 6, 16, 128, 192), (1, 32, 64, 64, 128), (2, 16, 16, 512, 512), (4, 16, 32, 16, 64),
    (2, 8, 16, 256, 128), (1, 2, 16, 64, 64),
]


@pytest.mark.parametrize('math', ['x3', 'x5', 'bf16', 'h2'])
@pytest.mark.parametrize('tune', [0, 'TUNE_WGRAD_R64', 'TUNE_W16_LAYOUT_2X2'])
@pytest.mark.parametrize('n,h,w,ci,co', WGRAD_PLANS)
def test_wgrad_slabs_fully_written(dev, math, tune, n, h, w, ci, co):
    """Slab coverage of the halo weight grads on every tile / split plan: with the workspace pre-filled with NaN, each
    slab element [split][row][tap * C + c] is written (no NaN left), and the finalized gradient matches fp64 at the
    arithmetic's accuracy.  One deterministic run per case (no repeat-until-fail)."""
    from multimodal_siamese_cd_amd import hip
    g = torch.Generator().manual_seed(n * h * w + ci + co)
    x = torch.randn(n, h, w, ci, generator=g)
    dy = torch.randn(n, h, w, co, generator=g)
    ref = torch.nn.grad.conv2d_weight(nchw(x).double(), (co, ci, 3, 3), nchw(dy).double(), padding=1)
    bits = 0 if tune == 0 else getattr(hip, tune)
    xd, dyd = x.to(dev), dy.to(dev)
    bx = by = None
    if math == 'h2':
        bx, by = xd.abs().max().reshape(1).clone(), dyd.abs().max().reshape(1).clone()
    with hip.conv_scope(math, bits):
        d, nsplit, nbytes = hip.wgrad_plan(hip.nhwc(dyd), hip.nhwc(xd), 1, hip.TAPS_3X3, None, by, bx)
        arith = hip.wgrad_arith(d)
        slabs = torch.full((nbytes // 4,), float('nan'), device=dev)
        hip.conv_wgrad(d, slabs)
    torch.cuda.synchronize()
    assert not torch.isnan(slabs).any(), f'{int(torch.isnan(slabs).sum())} slab elements never written ({arith})'
    dw = torch.empty(co, ci, 3, 3, device=dev)
    hip.wgrad_finalize(slabs, nsplit, co, 9, ci, 0, ci, dw)
    e = rel(dw, ref)
    assert e < (2e-2 if arith == 'bf16' else 2e-5), (arith, e)


@pytest.mark.parametrize('arith', ['f32', 'x3', 'bf16', 'h2'])
def test_batched_weight_pack_equals_standalone(dev, arith):
    """scd_pack_conv3x3_multi (LDS-staged 32-row x 64-column tiles, one launch for every job) writes the packed fp32
    layout and the split bytes the standalone pack + split would, for both layouts, on shapes with padded channels,
    row counts off the 32-row group and inner widths off the 64-column tile."""
    from multimodal_siamese_cd_amd import hip
    g = torch.Generator().manual_seed(7)
    shapes = [(64, 5, 16), (96, 64, 64), (48, 80, 80), (512, 512, 512), (64, 128, 128), (16, 32, 32)]
    ws = [(torch.randn(co, ci, 3, 3, generator=g) * 10 ** (2 * torch.rand(co, 1, 1, 1, generator=g) - 1)).to(dev)
          for co, ci, _ in shapes]
    jobs = []
    for (co, ci, cp), w in zip(shapes, ws):
        jobs.append((w, 0, cp))
        if ci == cp and co % 16 == 0:
            jobs.append((w, 1, ci))
    prev = hip.set_conv_math(arith)
    try:
        multi = hip.pack_conv3x3_multi(jobs)
        for (w, mode, cp), got in zip(jobs, multi):
            ref = hip.pack_conv3x3(w, mode, cp if mode == 0 else None)
            assert torch.equal(got, ref), (tuple(w.shape), mode)
            a, b = getattr(got, '_x3', None), getattr(ref, '_x3', None)
            assert (a is None) == (b is None), (tuple(w.shape), mode)
            if a is not None:
                rows, K = (w.shape[0], 9 * cp) if mode == 0 else (w.shape[1], 9 * w.shape[0])
                if arith == 'h2':  # two fp16 planes and the row scales; the rest of the buffer is not written
                    n = 2 * ((rows + 31) // 32 * 32) * K + 2 * ((rows + 31) // 32 * 32)
                    a, b = a[:n], b[:n]
                assert torch.equal(a, b), (tuple(w.shape), mode)
    finally:
        hip.set_conv_math(prev)


@pytest.mark.parametrize('math', ['h2', 'bf16'])
def test_wgrad_repeat_runs_identical(dev, math):
    """The surviving halo weight grads (the 16x16x32 kernels) run to run: eight launches per plan, each into a freshly
    NaN-filled slab workspace, write every slab element and produce bit-identical slabs (the closed round-2 hunt on
    the deleted 32x32 kernel, DESIGN 7: a block that skipped part of its slab range, or an LDS reuse race, would show
    here as a NaN or a changed bit).  A bounded check, not a repeat-until-fail hunt."""
    from multimodal_siamese_cd_amd import hip
    for n, h, w, ci, co in [(2, 16, 32, 128, 128), (3, 6, 16, 128, 192)]:
        g = torch.Generator().manual_seed(ci + co + h)
        xd = torch.randn(n, h, w, ci, generator=g).to(dev)
        dyd = torch.randn(n, h, w, co, generator=g).to(dev)
        bx = by = None
        if math == 'h2':
            bx, by = xd.abs().max().reshape(1).clone(), dyd.abs().max().reshape(1).clone()
        first = None
        with hip.conv_scope(math):
            for _ in range(8):
                d, nsplit, nbytes = hip.wgrad_plan(hip.nhwc(dyd), hip.nhwc(xd), 1, hip.TAPS_3X3, None, by, bx)
                slabs = torch.full((nbytes // 4,), float('nan'), device=dev)
                hip.conv_wgrad(d, slabs)
                torch.cuda.synchronize()
                assert not torch.isnan(slabs).any(), (n, h, w, ci, co)
                if first is None:
                    first = slabs.clone()
                else:
                    assert torch.equal(slabs, first), (n, h, w, ci, co)


@pytest.mark.parametrize('arith', ['x3', 'h2', 'bf16'])
def test_batched_convT_pack_equals_standalone(dev, arith):
    """scd_pack_convT2x2_multi (three launches for every job) writes the packed layouts and the split bytes (h2 where
    the format applies: 32-channel multiples; bf16x3 otherwise) of the one-weight pack_convT2x2, both modes, with more
    jobs than one launch holds (8)."""
    from multimodal_siamese_cd_amd import hip
    g = torch.Generator().manual_seed(9)
    shapes = [(512, 512), (256, 256), (128, 128), (64, 64), (48, 48), (16, 16), (96, 32), (32, 80), (8, 8)]
    jobs = []
    for ci, co in shapes:
        w = (torch.randn(ci, co, 2, 2, generator=g) * 10 ** (2 * torch.rand(ci, 1, 1, 1, generator=g) - 1)).to(dev)
        jobs += [(w, 0), (w, 1)]
    with hip.conv_scope(arith):
        multi = hip.pack_convT2x2_multi(jobs)
        for (w, mode), got in zip(jobs, multi):
            ref = hip.pack_convT2x2(w, mode)
            assert torch.equal(got, ref), (tuple(w.shape), mode)
            a, b = getattr(got, '_x3', None), getattr(ref, '_x3', None)
            assert (a is None) == (b is None), (tuple(w.shape), mode)
            if a is not None:
                ci, co = w.shape[0], w.shape[1]
                rows, K, taps = (4 * co, ci, 1) if mode == 0 else (ci, 4 * co, 4)
                if hip.h2_weight_format(K, taps):  # two fp16 planes and the row scales; the rest is not written
                    n = 2 * ((rows + 31) // 32 * 32) * K + 2 * ((rows + 31) // 32 * 32)
                    a, b = a[:n], b[:n]
                assert torch.equal(a, b), (tuple(w.shape), mode)
