"""The fused paths of the two-decoder and plain-encoder models (round 5, ABI 7) against the unfused paths they replace.

  fuse_plain_encoder  plain encoder levels (UNet, DualStreamUNet, WhateverNet2) write their activation into the decoder's
                      concat buffer and pool it in one pass (scd_bn_relu_pool_out mode 1): no bn_relu_apply, no skip
                      copy (the feature_grad_kernel-as-copy of DecoderFn)
  fuse_dualtask       DualTaskSiameseUNet's levels write the difference and the [t2; t1] semantic skip batch in one pass
                      (mode 2); the backward forms maxpool_bwd -/+ g_diff + g_sem inside the BatchNorm backward
                      (scd_bn_relu_backward_pooled2)
  dt_sem_batched      decoder_sem runs both dates as one 2B batch with per-date BatchNorm segments
  fuse_heads          DualStream's outc and WhateverNet(2)'s three heads as one launch over both decoders' last
                      BatchNorm + ReLU (scd_conv1x1_fwd_bn2 + scd_bn_relu_backward_head), no cat

Bit-identity runs under the split-bf16 arithmetic x3, which reads no operand bounds (under h2 the old dual-task path
bounds its differences by an absmax pass, the fused one by the BatchNorm statistics: a different power-of-two scale can
move the last bits).  The default (h2) fused paths are held to the reference fixtures by test_model_gpu.py.
"""
import pytest
import torch

from oracle.golden import Fixture

pytestmark = pytest.mark.gpu

OFF = dict(fuse_plain_encoder=False, fuse_dualtask=False, dt_sem_batched=False, fuse_heads=False)


@pytest.fixture(scope='module')
def dev():
    from multimodal_siamese_cd_amd import hip
    hip.load_library()
    return torch.device('cuda:0')


def _outs(o):
    return list(o) if isinstance(o, (tuple, list)) else [o]


def _run(fx, dev, opts, math='x3', eval_too=True):
    """One training step (forward, loss, backward) and an eval forward of the fixture's model under engine options."""
    from multimodal_siamese_cd_amd import engine, trainers
    from multimodal_siamese_cd_amd.utils import networks
    prev = engine.set_options(**opts)
    try:
        cfg = fx.package_cfg()
        cfg.MODEL.CONV_MATH = math
        net = networks.create_network(cfg)
        with torch.no_grad():
            for k, p in net.module.named_parameters():
                p.copy_(torch.from_numpy(fx.params0[k]))
        net = net.to(dev).train()
        batch = {k: v.to(dev) for k, v in fx.batch().items()}
        out = net(batch['x_t1'], batch['x_t2'])
        loss = trainers.step_loss(cfg, out, batch)
        loss.backward()
        ev = []
        if eval_too:
            net.eval()
            with torch.no_grad():
                ev = [o.cpu() for o in _outs(net(batch['x_t1'], batch['x_t2']))]
        torch.cuda.synchronize()
        return dict(out=[o.detach().cpu() for o in _outs(out)], loss=loss.item(), eval=ev,
                    grads={k: p.grad.cpu() for k, p in net.module.named_parameters() if p.grad is not None},
                    bufs={k: b.cpu() for k, b in net.module.named_buffers()})
    finally:
        engine.set_options(**prev)


def _head_weight(k):
    return k.startswith('outc') and k.endswith('.weight')


def _pre_bn_bias(k):  # a conv bias feeding a train-mode BatchNorm: true gradient 0, float noise either way
    return k.endswith('conv.0.bias') or k.endswith('conv.3.bias')


@pytest.mark.parametrize('name', ['unet_t8-16', 'dualstream_t8-16', 'dualstream_t32-64', 'dualstream_t8-16_odd',
                                  'dualstream_t6-12', 'whatevernet2_t8-16', 'whatevernet_t8-16', 'dtsiamese_t8-16',
                                  'dtsiamese_t32-64'])
def test_fused_forward_bit_identical(dev, name):
    """Logits (train and eval), loss and BatchNorm buffers of the fused paths equal the unfused ones bit for bit."""
    fx = Fixture(name)
    on = _run(fx, dev, {})
    off = _run(fx, dev, OFF)
    assert on['loss'] == off['loss']
    for a, b in zip(on['out'] + on['eval'], off['out'] + off['eval']):
        assert torch.equal(a, b)
    for k in off['bufs']:
        assert torch.equal(on['bufs'][k], off['bufs'][k]), k


@pytest.mark.parametrize('name', ['unet_t8-16', 'dualstream_t8-16', 'dualstream_t32-64', 'dualstream_t8-16_odd',
                                  'whatevernet2_t8-16', 'dtsiamese_t8-16', 'dtsiamese_t32-64'])
def test_fused_backward_bit_identical(dev, name):
    """Every gradient of the fused paths equals the unfused one bit for bit where the fused backward sums the same
    terms in the same order: the plain and dual-task encoders (the second skip gradient is added to the difference
    gradient first, as autograd sums the two before the level's backward), a single fusion head (DualStream).  The
    head weights come from the BatchNorm backward's pass (1e-6: the products' rounding may contract differently), and
    WhateverNet2's stream-1/2 decoders, read by two heads, form sum_k g_k w_k in one fma chain where autograd rounds each
    head's input gradient before adding them (1e-5)."""
    fx = Fixture(name)
    opts = {'dt_sem_batched': False}
    on = _run(fx, dev, opts, eval_too=False)
    off = _run(fx, dev, OFF, eval_too=False)
    assert on['grads'].keys() == off['grads'].keys()
    two_heads = fx.model_type == 'whatevernet2'
    for k in off['grads']:
        a, b = on['grads'][k], off['grads'][k]
        if _head_weight(k) or (two_heads and 'stream' in k):
            if _pre_bn_bias(k):  # ~0 both ways: judged against its weight's gradient
                w = off['grads'][k.replace('.bias', '.weight')]
                assert float((a - b).abs().max()) < 1e-5 * float(w.abs().max()), k
                continue
            err = float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))
            assert err < (1e-5 if two_heads else 1e-6), (k, err)
        else:
            assert torch.equal(a, b), k


@pytest.mark.parametrize('name', ['dtsiamese_t8-16', 'dtsiamese_t32-64'])
def test_dualtask_sem_batch_matches_two_calls(dev, name):
    """decoder_sem over the [t2; t1] batch with per-date BatchNorm segments vs two calls on the halves: logits, loss and
    running statistics bit-identical (per-image convs, per-segment statistics from the same tile records in the same
    order), gradients equal up to the order the two dates' weight-grad terms are summed (1e-5)."""
    fx = Fixture(name)
    one = _run(fx, dev, {'dt_sem_batched': True})
    two = _run(fx, dev, {'dt_sem_batched': False})
    assert one['loss'] == two['loss']
    for a, b in zip(one['out'] + one['eval'], two['out'] + two['eval']):
        assert torch.equal(a, b)
    for k in two['bufs']:
        assert torch.equal(one['bufs'][k], two['bufs'][k]), k
    for k in two['grads']:
        a, b = one['grads'][k], two['grads'][k]
        if _pre_bn_bias(k):
            w = two['grads'][k.replace('.bias', '.weight')]
            assert float((a - b).abs().max()) < 1e-5 * float(w.abs().max()), k
            continue
        err = float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))
        assert err < 1e-5, (k, err)


@pytest.mark.parametrize('name', ['whatevernet_t8-16', 'whatevernet2_t8-16', 'dualstream_t8-16', 'dtsiamese_t8-16'])
def test_fused_paths_take_no_copies(dev, name, monkeypatch):
    """The fused forwards launch no skip / cat copy (scd_feature_grad used as a copy), no bn_relu_apply for an encoder
    level or a head's input (a DoubleConv's inner activation is materialised where its second conv cannot read it
    through the BatchNorm, both ways) and no separate head per output (one scd_conv1x1_fwd_bn2 launch for the
    two-decoder models)."""
    from multimodal_siamese_cd_amd import hip
    counts = []
    for opts in ({'dt_sem_batched': False}, OFF):  # decoder_sem as two calls both ways: the same decoder launches
        calls = {}
        with monkeypatch.context() as m:
            for fn in ('feature_grad', 'bn_relu_apply', 'conv1x1_fwd', 'conv1x1_fwd_bn', 'conv1x1_fwd_bn2',
                       'bn_relu_pool_out', 'siamese_diff', 'maxpool2_fwd'):
                orig = getattr(hip, fn)

                def wrap(*a, _fn=fn, _orig=orig, _c=calls, **k):
                    _c[_fn] = _c.get(_fn, 0) + 1
                    return _orig(*a, **k)
                m.setattr(hip, fn, wrap)
            fx = Fixture(name)
            _run(fx, dev, opts, math='h2', eval_too=False)
        counts.append(calls)
    calls, off = counts
    levels = len(fx.cfg['TOPOLOGY']) + 1
    saved = {'dualstreamunet': 2 * (levels + 1), 'whatevernet2': 2 * (levels + 1), 'whatevernet': 2,
             'dtsiameseunet': levels}[fx.model_type]  # encoder levels + decoder outputs materialised by the old paths
    assert off.get('bn_relu_apply', 0) - calls.get('bn_relu_apply', 0) == saved, (calls, off)
    assert calls.get('feature_grad', 0) == 0, calls
    assert calls.get('siamese_diff', 0) == 0 and calls.get('maxpool2_fwd', 0) == 0, calls
    if fx.model_type != 'whatevernet':  # its Siamese streams take scd_bn_relu_pool_diff
        assert calls.get('bn_relu_pool_out', 0) > 0, calls
    if fx.model_type in ('whatevernet', 'whatevernet2', 'dualstreamunet'):
        assert calls.get('conv1x1_fwd_bn2', 0) == 1 and calls.get('conv1x1_fwd', 0) == 0, calls


# ------------------------------------------------------------------------------------------------
# kernel level
# ------------------------------------------------------------------------------------------------
def _bn_relu_ref(y, sc, sh, nseg):
    """max(fmaf(y, scale, shift), 0) per segment: the product is exact in fp64, one rounding to fp32 after the add."""
    n = y.shape[0]
    c = y.shape[3]
    seg = torch.arange(n, device=y.device) // (n // nseg)
    z = y.double() * sc.double().view(nseg, c)[seg][:, None, None] + sh.double().view(nseg, c)[seg][:, None, None]
    return torch.clamp_min(z.float(), 0.0)


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('mode', [1, 2])
def test_bn_relu_pool_out_matches_materialised(dev, dtype, mode):
    """scd_bn_relu_pool_out modes 1 and 2 equal materialising a = relu(bn(y)) in the storage type and running the copy,
    difference and MaxPool2d on it (values and argmax bytes), into concat-buffer slices, with and without pooling."""
    from multimodal_siamese_cd_amd import hip
    from multimodal_siamese_cd_amd.hip import nhwc
    g = torch.Generator(device=dev).manual_seed(5)
    n, h, w, c, extra = 4, 10, 12, 32, 8
    nseg = 2
    y = torch.randn((n, h, w, c), device=dev, generator=g).to(dtype)
    y[0, 0, 0, :4] = y[0, 0, 1, :4]  # exact ties in a pooling window
    sc = torch.rand(nseg * c, device=dev, generator=g) + 0.5
    sh = torch.randn(nseg * c, device=dev, generator=g) * 0.3
    a = _bn_relu_ref(y, sc, sh, nseg).to(dtype)  # the stored activation
    b = n // 2
    for pool in (True, False):
        nxt = torch.empty((n, h // 2, w // 2, c), device=dev, dtype=dtype) if pool else None
        idx = torch.empty((n, h // 2, w // 2, c), device=dev, dtype=torch.uint8) if pool else None
        if mode == 1:
            buf = torch.full((n, h, w, c + extra), 7.0, device=dev, dtype=dtype)
            hip.bn_relu_pool_out(nhwc(y), nseg, sc, sh, hip.POOL_COPY, hip._NULL, nhwc(buf, 0, c),
                                 nhwc(nxt) if pool else hip._NULL, idx)
            assert torch.equal(buf[..., :c], a) and bool((buf[..., c:] == 7).all())
        else:
            bufc = torch.full((b, h, w, c + extra), 7.0, device=dev, dtype=dtype)
            bufs = torch.full((n, h, w, c + extra), 7.0, device=dev, dtype=dtype)
            hip.bn_relu_pool_out(nhwc(y), 2, sc, sh, hip.POOL_DIFF_COPY, nhwc(bufc, 0, c), nhwc(bufs, 0, c),
                                 nhwc(nxt) if pool else hip._NULL, idx)
            assert torch.equal(bufc[..., :c], (a[b:].float() - a[:b].float()).to(dtype))
            assert torch.equal(bufs[..., :c], torch.cat([a[b:], a[:b]]))
            assert bool((bufc[..., c:] == 7).all()) and bool((bufs[..., c:] == 7).all())
        if pool:
            ref = torch.nn.functional.max_pool2d(a.float().permute(0, 3, 1, 2), 2, return_indices=True)
            assert torch.equal(nxt.float(), ref[0].permute(0, 2, 3, 1))
            # argmax byte k = (row in window) * 2 + (col in window), first max wins as aten's
            r, q = ref[1] // w, ref[1] % w
            want = ((r % 2) * 2 + (q % 2)).permute(0, 2, 3, 1).to(torch.uint8)
            assert torch.equal(idx, want)


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
def test_bn_relu_backward_pooled2_matches_materialised(dev, dtype):
    """The dual-task pooled BatchNorm backward (skip_mode 2: maxpool_bwd(gy) + (-/+ g_diff + g_sem[swapped])) equals the
    plain-skip pooled backward (skip_mode 0) fed the materialised skip gradient -/+ g_diff + g_sem[swapped] -- what the
    unfused dual-task path hands it after autograd's sum -- bit for bit in fp32 (the pair kernel writes the per-chunk
    records of the per-image walk); in bf16 the materialised skip is rounded once more (tolerance)."""
    from multimodal_siamese_cd_amd import hip
    from multimodal_siamese_cd_amd.hip import nhwc
    g = torch.Generator(device=dev).manual_seed(11)
    n, h, w, c = 4, 8, 12, 32
    b = n // 2
    y = torch.randn((n, h, w, c), device=dev, generator=g).to(dtype)
    gy = torch.randn((n, h // 2, w // 2, c), device=dev, generator=g).to(dtype)
    idx = torch.randint(0, 4, (n, h // 2, w // 2, c), device=dev, generator=g, dtype=torch.uint8)
    gd = torch.randn((b, h, w, c), device=dev, generator=g).to(dtype)
    gs = torch.randn((n, h, w, c), device=dev, generator=g).to(dtype)
    smean = torch.randn(2 * c, device=dev, generator=g) * 0.1
    sinv = torch.rand(2 * c, device=dev, generator=g) + 0.5
    gamma = torch.rand(c, device=dev, generator=g) + 0.5
    scale = torch.rand(2 * c, device=dev, generator=g) + 0.5
    shift = torch.randn(2 * c, device=dev, generator=g) * 0.3
    sgn = torch.cat([-torch.ones(b), torch.ones(b)]).to(dev)[:, None, None, None]
    skip = (sgn * torch.cat([gd, gd]).float() + torch.cat([gs[b:], gs[:b]]).float()).to(dtype)
    outs = []
    for fused in (True, False):
        dy = torch.empty_like(y)
        dg, db, dbias = (torch.empty(c, device=dev) for _ in range(3))
        ws = torch.empty(hip.bn_workspace_bytes(n, h, w, c, 2), device=dev, dtype=torch.uint8)
        if fused:
            hip.bn_relu_backward_pooled2(nhwc(y), nhwc(gy), idx, nhwc(gd), 2, nhwc(gs), 2, smean, sinv, gamma, scale,
                                         shift, dg, db, dbias, nhwc(dy), ws)
        else:
            hip.bn_relu_backward_pooled(nhwc(y), nhwc(gy), idx, nhwc(skip), 0, 2, smean, sinv, gamma, scale, shift,
                                        dg, db, dbias, nhwc(dy), ws)
        outs.append((dy, dg, db, dbias))
    if dtype == torch.float32:
        for a, b_ in zip(*outs):
            assert torch.equal(a, b_)
    else:
        for a, b_ in zip(outs[0][:3], outs[1][:3]):
            err = float((a.float() - b_.float()).abs().max() / b_.float().abs().max())
            assert err < 2e-2, err
        # the conv-bias grad cancels to ~0 (a pre-BN bias): judged against the sum of |dy|
        assert ((outs[0][3] - outs[1][3]).abs() <= 1e-2 * outs[1][0].float().abs().sum(dim=(0, 1, 2))).all()


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
def test_two_source_heads_equal_cat(dev, dtype):
    """scd_conv1x1_fwd_bn2 over two sources (their own coefficients, three stacked heads with zero blocks) equals the
    single-source head over the materialised concatenation bit for bit (same pieces, chains and tree), and a torch fp64
    reference within fp32 rounding."""
    from multimodal_siamese_cd_amd import hip
    from multimodal_siamese_cd_amd.hip import nhwc
    g = torch.Generator(device=dev).manual_seed(3)
    n, h, w, c = 3, 16, 20, 64
    ya = torch.randn((n, h, w, c), device=dev, generator=g).to(dtype)
    yb = torch.randn((n, h, w, c), device=dev, generator=g).to(dtype)
    sa, ha, sb, hb = (torch.randn(c, device=dev, generator=g) for _ in range(4))
    wt = torch.randn((3, 2 * c), device=dev, generator=g)
    wt[1, c:] = 0  # head "stream 1" reads a only
    wt[2, :c] = 0  # head "stream 2" reads b only
    bias = torch.randn(3, device=dev, generator=g)
    out2 = torch.empty((n, 3, h, w), device=dev)
    hip.conv1x1_fwd_bn2(nhwc(ya), sa, ha, nhwc(yb), sb, hb, 1, wt, bias, 3, out2)
    cat = torch.cat([_bn_relu_ref(ya, sa, ha, 1), _bn_relu_ref(yb, sb, hb, 1)], dim=3).contiguous()
    ref = (torch.einsum('nhwc,oc->nohw', cat.double(), wt.double()) + bias.double()[None, :, None, None]).float()
    assert float((out2 - ref).abs().max() / ref.abs().max()) < 1e-5
    if dtype == torch.float32:  # the single-source launch over the materialised fp32 cat
        out1 = torch.empty_like(out2)
        hip.conv1x1_fwd(nhwc(cat), wt, bias, 3, out1)
        assert torch.equal(out1, out2)
        one = torch.empty((n, 1, h, w), device=dev)  # stream-1 head alone over a (half the lanes): same bits
        hip.conv1x1_fwd_bn(nhwc(ya), sa, ha, 1, wt[1:2, :c].contiguous(), bias[1:2], 1, one)
        assert torch.equal(one[:, 0], out2[:, 1])


def _step_grads(cfg, dev, opts, params0, b):
    """One training step of a freshly built model with the given parameters; returns {name: grad} (CPU)."""
    from multimodal_siamese_cd_amd import engine, trainers
    from multimodal_siamese_cd_amd.utils import networks
    prev = engine.set_options(**opts)
    try:
        net = networks.create_network(cfg)
        with torch.no_grad():
            for k, p in net.module.named_parameters():
                p.copy_(params0[k])
        net = net.to(dev).train()
        loss = trainers.step_loss(cfg, net(b['x_t1'], b['x_t2']), b)
        loss.backward()
        torch.cuda.synchronize()
        return {k: p.grad.cpu() for k, p in net.module.named_parameters() if p.grad is not None}
    finally:
        engine.set_options(**prev)


@pytest.mark.parametrize('config,math', [('baseline_siamese', 'bf16'), ('baseline_dualstream', 'bf16'),
                                         ('dtsiamese', 'bf16'), ('baseline_siamese', 'h2')])
def test_bn_bwd_in_wgrad_matches_apply_path(dev, config, math):
    """ABI 8: plain BatchNorm backwards formed inside the weight grads (engine option bn_bwd_in_wgrad, the weight grad
    stores dy for the data grad) against the apply pass they replace, on models with 64- and 128-channel layers
    (TOPOLOGY [64, 128, 256], 64^2 crops).  bf16: every weight, gamma and beta gradient bit for bit (dy is formed with
    bn_bwd_apply's expression and rounding; the weight grads read the same operands).  The conv biases before a
    BatchNorm (true gradient 0) come from the statistics instead of a sum over dy: both are rounding noise, judged
    against the weight's gradient.  h2: the weight grad scales dy by a bound from the statistics rather than its
    max, which moves only values near the fp16 subnormal range: within 1e-6."""
    from multimodal_siamese_cd_amd.utils import datasets, experiment_manager, networks
    cfg = experiment_manager.load_cfg(config)
    cfg.MODEL.TOPOLOGY = [64, 128, 256]
    cfg.MODEL.CONV_MATH = math
    cfg.AUGMENTATION.CROP_SIZE = 64
    torch.manual_seed(3)
    params0 = {k: p.detach().clone() for k, p in networks.create_network(cfg).module.named_parameters()}
    b = datasets.synthetic_batch(cfg, 4, dev, torch.Generator(device=dev).manual_seed(11))
    on = _step_grads(cfg, dev, {'bn_bwd_in_wgrad': 128}, params0, b)
    off = _step_grads(cfg, dev, {'bn_bwd_in_wgrad': 0}, params0, b)
    assert on.keys() == off.keys()
    for k in off:
        a, r = on[k], off[k]
        if _pre_bn_bias(k):
            w = off[k.replace('.bias', '.weight')]
            assert float((a - r).abs().max()) < 1e-4 * float(w.abs().max()), k
        elif math == 'bf16':
            assert torch.equal(a, r), k
        else:
            err = float((a - r).abs().max() / r.abs().max().clamp_min(1e-30))
            assert err < 1e-6, (k, err)
