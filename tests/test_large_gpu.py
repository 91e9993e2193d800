"""Operands of 2 GiB and more (the Siamese level-0 maps at bs=64: 128 x 256^2 x 64 fp32 = 2.1 GB).

The buffer-load kernels use 32-bit byte offsets, so scd_conv_igemm / scd_conv_wgrad split such convs into image
chunks (conv_f32.hip image_chunk).  Per-image work is independent, so the chunked forward (with fused BatchNorm
statistics and input transform) must be bit-identical to launching the image halves by hand; the weight grad of
the whole batch must equal the sum of the halves' weight grads up to fp32 summation order (1e-5).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

N, H, W, C, CO = 130, 256, 256, 64, 64  # 130 * 256^2 * 64 * 4 B = 2.18 GB per map


@pytest.fixture(scope='module')
def dev():
    from multimodal_siamese_cd_amd import hip
    hip.load_library()
    d = torch.device('cuda:0')
    hip.ensure_device(torch.empty(1, device=d))
    return d


@pytest.fixture(scope='module')
def big(dev):
    g = torch.Generator(device=dev).manual_seed(5)
    x = torch.randn(N, H, W, C, device=dev, generator=g)
    assert x.numel() * 4 >= 2 ** 31
    return x


@pytest.mark.parametrize('math', ['x3', 'bf16', 'h2'])
def test_igemm_over_2gib_matches_image_halves(dev, big, math):
    from multimodal_siamese_cd_amd import hip
    prev = hip.set_conv_math(math)
    ub = torch.full((1,), 64.0, device=dev) if math == 'h2' else None  # h2: a (loose) bound of the BN'd input
    try:
        g = torch.Generator(device=dev).manual_seed(6)
        wt = torch.randn(CO, C, 3, 3, device=dev, generator=g) / 24
        b = torch.randn(CO, device=dev, generator=g)
        sc = torch.rand(2 * C, device=dev, generator=g) + 0.5
        sh = torch.randn(2 * C, device=dev, generator=g)
        wpk = hip.pack_conv3x3(wt, 0)
        y = torch.empty(N, H, W, CO, device=dev)
        ntiles, tpx = hip.igemm_stat_tiles(hip.nhwc(big), H, W, 1, hip.TAPS_3X3, wpk, CO, hip.nhwc(y), src_bound=ub)
        assert ntiles > 0, 'fused statistics must stay available above 2 GiB'
        bn = (sc, sh, 2)
        assert hip.igemm_input_bn_supported(hip.nhwc(big), H, W, 1, hip.TAPS_3X3, wpk, CO, hip.nhwc(y), bn, ub)
        assert hip.igemm_arith(hip.nhwc(big), H, W, 1, hip.TAPS_3X3, wpk, CO, hip.nhwc(y), src_bound=ub) == math
        rec = torch.empty(ntiles * CO * 2, device=dev)
        hip.conv_igemm(hip.nhwc(big), H, W, 1, hip.TAPS_3X3, wpk, CO, b, hip.nhwc(y), stat_rec=rec, in_bn=bn,
                       src_bound=ub)
        half = N // 2  # one BatchNorm segment each
        tpi = ntiles // N
        for i in range(2):
            xs = big[i * half:(i + 1) * half]
            ys = torch.empty(half, H, W, CO, device=dev)
            rs = torch.empty(tpi * half * CO * 2, device=dev)
            hip.conv_igemm(hip.nhwc(xs), H, W, 1, hip.TAPS_3X3, wpk, CO, b, hip.nhwc(ys), stat_rec=rs,
                           in_bn=(sc[i * C:(i + 1) * C], sh[i * C:(i + 1) * C], 1), src_bound=ub)
            assert torch.equal(ys, y[i * half:(i + 1) * half])
            assert torch.equal(rs, rec[i * tpi * half * CO * 2:(i + 1) * tpi * half * CO * 2])
    finally:
        hip.set_conv_math(prev)


@pytest.mark.parametrize('math', ['x3', 'bf16', 'h2'])
def test_wgrad_over_2gib_matches_sum_of_halves(dev, big, math):
    from multimodal_siamese_cd_amd import hip
    prev = hip.set_conv_math(math)
    ub = torch.full((1,), 16.0, device=dev) if math == 'h2' else None  # h2: bound of the N(0, 1) operands
    try:
        g = torch.Generator(device=dev).manual_seed(8)
        dy = torch.randn(N, H, W, CO, device=dev, generator=g)

        def wgrad(rows, src):
            d, nsplit, nbytes = hip.wgrad_plan(hip.nhwc(rows), hip.nhwc(src), 1, hip.TAPS_3X3, None, ub, ub)
            assert hip.wgrad_arith(d) == math
            slabs = torch.empty(nbytes // 4, device=dev)
            hip.conv_wgrad(d, slabs)
            dw = torch.empty(CO, C, 3, 3, device=dev)
            hip.wgrad_finalize(slabs, nsplit, CO, 9, C, 0, C, dw)
            return dw

        full = wgrad(dy, big)
        half = N // 2
        parts = wgrad(dy[:half], big[:half]).double() + wgrad(dy[half:], big[half:]).double()
        err = ((full.double() - parts).abs().max() / parts.abs().max()).item()
        assert err < 1e-5, err  # 8.5 M-term fp32 sums split differently
    finally:
        hip.set_conv_math(prev)


def test_wgrad_rows_bn_over_2gib_stores_dy(dev, big):
    """ABI 8 on image chunks: the halo weight grad forming a plain BatchNorm backward's dy (rows_y) and storing it
    (rows_out) over a > 2 GiB batch with two BatchNorm segments is split into chunks like any weight grad; the stored dy
    must equal scd_bn_relu_backward's bit for bit and its bound the exact max.  The weight grad equals the
    materialised dy's up to fp32 summation order: with the rows transform a chunk keeps whole BatchNorm segments
    (65 images here), without it the chunks are as large as 2 GiB allows, so the K-splits differ (bf16
    arithmetic, fp32 storage, R = C = 64)."""
    from multimodal_siamese_cd_amd import hip
    prev = hip.set_conv_math('bf16')
    try:
        g = torch.Generator(device=dev).manual_seed(9)
        y = torch.randn(N, H, W, CO, device=dev, generator=g) * 2 + 0.3
        da = torch.randn(N, H, W, CO, device=dev, generator=g)
        nseg = 2
        gamma = torch.rand(CO, device=dev, generator=g) + 0.5
        beta = torch.randn(CO, device=dev, generator=g)
        smean, sinv, scale, shift = (torch.empty(nseg * CO, device=dev) for _ in range(4))
        ws = torch.empty(hip.bn_workspace_bytes(N, H, W, CO, nseg), dtype=torch.uint8, device=dev)
        hip.bn_train_stats(hip.nhwc(y), nseg, gamma, beta, 1e-5, 0.1, False, None, None, smean, sinv, scale, shift,
                           ws)
        dy = torch.empty_like(y)
        o = [torch.empty(CO, device=dev) for _ in range(3)]
        hip.bn_relu_backward(hip.nhwc(y), hip.nhwc(da), nseg, smean, sinv, gamma, scale, shift, *o, hip.nhwc(dy), ws)
        coef = torch.empty(nseg * CO * 2, device=dev)
        q = [torch.empty(CO, device=dev) for _ in range(3)]
        hip.bn_relu_backward_coef(hip.nhwc(y), hip.nhwc(da), nseg, smean, sinv, gamma, scale, shift, None, 0, coef,
                                  *q, ws)
        out = torch.empty_like(y)
        ob = torch.zeros(1, device=dev)

        def wgrad(rows, rows_bn=None, rows_out=None):
            d, nsplit, nbytes = hip.wgrad_plan(hip.nhwc(rows), hip.nhwc(big), 1, hip.TAPS_3X3, rows_bn=rows_bn,
                                               rows_out=rows_out, rows_out_bound=ob)
            assert hip.wgrad_arith(d) == 'bf16'
            slabs = torch.empty(nbytes // 4, device=dev)
            hip.conv_wgrad(d, slabs)
            dw = torch.empty(CO, C, 3, 3, device=dev)
            hip.wgrad_finalize(slabs, nsplit, CO, 9, C, 0, C, dw)
            return dw

        ref = wgrad(dy)
        fused = wgrad(da, (hip.nhwc(y), nseg, smean, sinv, gamma, scale, shift, coef), hip.nhwc(out))
        torch.cuda.synchronize()
        assert torch.equal(out, dy)
        assert ob.item() == dy.abs().max().item()
        err = ((fused.double() - ref.double()).abs().max() / ref.double().abs().max()).item()
        assert err < 1e-5, err
    finally:
        hip.set_conv_math(prev)
