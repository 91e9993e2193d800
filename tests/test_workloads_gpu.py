"""Every shipped BASELINE workload against the oracle on the production kernels (MI355X).

The model is built only through the drop-in surface (utils.networks.create_network with the workload's config), so
it runs the arithmetic its config selects (MODEL.PRECISION fp32 -> h2, bf16 -> bf16); every conv launch is checked
to run that arithmetic wherever the library's kernels take it.

fp32 workloads (h2): against the fp64 oracle following the GPU forward's own ReLU / MaxPool branches (tests/_parity.py
branch matching): outputs within 1e-4 (north_star's logits bar), change masks bit-exact outside the |logit| < 1e-4
max band, loss within 1e-5, BatchNorm running statistics within 1e-5, every gradient tensor within 1e-3 max-relative.

bf16 workloads: bf16 roundings amplify through depth, so no bf16 implementation matches another to fp32 precision at
model level (the kernel tests pin the arithmetic exactly).  Outputs within 3e-2 of the fp32 oracle and closer to an
oracle with the bf16 conv arithmetic emulated than to the fp32 one; loss within 1e-2; every weight gradient's cosine
similarity to the fp32 oracle's at most 0.05 below what the bf16-emulating oracle itself reaches, and > 0.85 (the
emulating oracle itself reaches 0.897 on the WhateverNet BatchNorm shifts of the deepest levels at 512x512) wherever
the emulating oracle reaches 0.9 -- at the shipped bs=64 the large-map ConvTranspose bias sums do not (round 6).

Sizes: the workloads' own tiles and topologies ([64, 128, 256, 512], 256x256; WhateverNet 512x512) at bs=2, the
headline baseline_siamese at its bench batch, bs=32 (the BatchNorm-derived h2 bounds grow with the batch), and every
workload at its shipped batch, forward and backward (siamese and dtsiamese bs=64, dual-stream bs=64, MMCR bs=4).
"""
import contextlib

import numpy as np
import pytest
import torch

from _parity import bf16_conv_oracle, branch_matched_reference, check_branch_matched, mask_mismatch, record_arith, rel

pytestmark = pytest.mark.gpu

FULL = [64, 128, 256, 512]


@pytest.fixture(scope='module')
def dev():
    from multimodal_siamese_cd_amd import hip
    hip.load_library()
    d = torch.device('cuda:0')
    hip.ensure_device(torch.empty(1, device=d))
    return d


def _cfg(config, model, topo, **model_kw):
    """The shipped config file (configs/<config>.yaml), its model type and topology, plus overrides."""
    from multimodal_siamese_cd_amd.utils import experiment_manager as em
    cfg = em.load_cfg(config)
    cfg.MODEL.TYPE = model
    cfg.MODEL.TOPOLOGY = list(topo)
    for k, v in model_kw.items():
        cfg.MODEL[k] = v
    return cfg


def _ocfg(cfg):
    return dict(TYPE=cfg.MODEL.TYPE, TOPOLOGY=list(cfg.MODEL.TOPOLOGY), IN_CHANNELS=cfg.MODEL.IN_CHANNELS,
                OUT_CHANNELS=cfg.MODEL.OUT_CHANNELS, S1_BANDS=list(cfg.DATALOADER.S1_BANDS),
                S2_BANDS=list(cfg.DATALOADER.S2_BANDS))


def _outs(o):
    return list(o) if isinstance(o, (tuple, list)) else [o]


def _gpu_step(cfg, P, batch, dev, monkeypatch, trace_bn=True):
    """One training step of the drop-in model on the GPU: (outputs, loss, grads, state_dict, launches, arithmetic,
    (BatchNorm trace, module)).  trace_bn=False: no BatchNorm trace (it clones every conv output: too much device memory
    at the shipped batches)."""
    from multimodal_siamese_cd_amd import engine, trainers
    from multimodal_siamese_cd_amd.utils import networks
    net = networks.create_network(cfg)
    with torch.no_grad():
        for k, p in net.module.named_parameters():
            p.copy_(P[k])
    net.to(dev).train()
    seen = record_arith(monkeypatch, dev)
    b = {k: v.to(dev) for k, v in batch.items()}
    with (engine.trace_bn() if trace_bn else contextlib.nullcontext([])) as trace:
        out = net(b['x_t1'], b['x_t2'])
    loss = trainers.step_loss(cfg, out, b)
    loss.backward()
    monkeypatch.undo()
    torch.cuda.synchronize()
    return ([o.detach().cpu() for o in _outs(out)], loss.item(),
            {k: p.grad.detach().cpu() for k, p in net.module.named_parameters() if p.grad is not None},
            {k: v.detach().cpu() for k, v in net.module.state_dict().items()}, seen, net.module.conv_math,
            (trace, net.module))


def _oracle_step(cfg, P, batch, dtype, alpha=0.5):
    from oracle import siamese_oracle as O
    ocfg = _ocfg(cfg)
    model = cfg.MODEL.TYPE
    shapes = O.param_shapes(model, ocfg)
    Pr = {k: v.detach().to(dtype).clone().requires_grad_(True) for k, v in P.items()}
    B = {k: (v.to(dtype) if v.is_floating_point() else v.clone()) for k, v in O.fresh_buffers(shapes).items()}
    bt = {k: (v.to(dtype) if v.is_floating_point() else v) for k, v in batch.items()}
    out = O.forward(model, Pr, B, bt['x_t1'], bt['x_t2'], ocfg, True)
    loss = O.step_loss(model, out, bt, alpha)
    loss.backward()
    return ([o.detach() for o in _outs(out)], loss.item(),
            {k: v.grad for k, v in Pr.items() if v.grad is not None}, B)


def _setup(cfg, batch_size, size, labeled=None, seed=7):
    from oracle import siamese_oracle as O
    ocfg = _ocfg(cfg)
    P = O.deterministic_params(O.param_shapes(cfg.MODEL.TYPE, ocfg), seed)
    batch = O.synthetic_batch(ocfg, batch_size, size, seed + 1, labeled)
    return P, batch


def _check_routing(seen, math, require=True):
    """Every conv launch runs the arithmetic it would run with bounds on every operand (no h2-capable conv left on
    x3 for want of a bound), and (`require`) at least one runs `math`."""
    assert seen, 'no conv launches recorded'
    assert all(s[4] == s[5] for s in seen), [s for s in seen if s[4] != s[5]]
    n = sum(s[4] == math for s in seen)
    print(f'{n} of {len(seen)} conv launches run {math}')
    assert n > 0 or not require


FP32_WORKLOADS = [
    # id, config file, model, topology, tile, batch
    ('dtsiamese', 'dtsiamese', 'dtsiameseunet', FULL, 256, 2),
    ('baseline_siamese_bs32', 'baseline_siamese', 'siameseunet', FULL, 256, 32),
    # ConvTranspose inputs of 24 / 40 channels (c % 16 == 8): no split-kernel epilogue bound, an absmax pass instead
    ('siamese_t24-32', 'baseline_siamese', 'siameseunet', [24, 32], 32, 2),
    ('unet_t16-40', 'baseline_siamese', 'unet', [16, 40], 32, 2),
]


@pytest.mark.parametrize('wid,config,model,topo,size,bs', FP32_WORKLOADS, ids=[w[0] for w in FP32_WORKLOADS])
def test_fp32_workload_matches_oracle(dev, monkeypatch, wid, config, model, topo, size, bs):
    cfg = _cfg(config, model, topo, PRECISION='fp32')
    P, batch = _setup(cfg, bs, size)
    outs, loss, grads, sd, seen, math, (trace, module) = _gpu_step(cfg, P, batch, dev, monkeypatch)
    assert math == 'h2'
    _check_routing(seen, 'h2', require=min(topo) >= 32)  # the h2 halo kernels need >= 64 output channels
    from oracle import siamese_oracle as O
    ocfg = _ocfg(cfg)
    ref_B = O.fresh_buffers(O.param_shapes(model, ocfg))
    ref_out, ref_loss, ref_g = branch_matched_reference(model, P, batch, ocfg, trace, module,
                                                        lambda o, bt: O.step_loss(model, o, bt, 0.5), buffers=ref_B)
    for i, (o, r) in enumerate(zip(outs, _outs(ref_out))):
        e = rel(o, r)
        print(f'output {i}: rel err vs the fp64 oracle {e:.2e}')
        assert e < 1e-4
        assert mask_mismatch(o.numpy(), r.detach().numpy()) == 0
    assert abs(loss - ref_loss.item()) < 1e-5
    for k, v in ref_B.items():
        if k.endswith('running_mean') or k.endswith('running_var'):
            assert rel(sd[k], v) < 1e-5, k
        elif k.endswith('num_batches_tracked'):
            assert int(sd[k]) == int(v), k
    bad = check_branch_matched(grads, ref_g, list(grads), 1e-3)
    assert not bad, bad


BF16_WORKLOADS = [
    # id, config file, model, topology, tile, batch, labelled samples
    # (siamese_mmcr_alpha0500 runs at its shipped batch, bs=4, in test_mmcr_shipped_batch: one oracle pass of each kind
    # there instead of a bs=2 pass here as well)
    ('baseline_dualstream', 'baseline_dualstream', 'dualstreamunet', FULL, 256, 2, None),
]


@pytest.mark.parametrize('wid,config,model,topo,size,bs,labeled', BF16_WORKLOADS, ids=[w[0] for w in BF16_WORKLOADS])
def test_bf16_workload_matches_oracle(dev, monkeypatch, wid, config, model, topo, size, bs, labeled):
    cfg = _cfg(config, model, topo)
    assert str(cfg.MODEL.PRECISION) == 'bf16'
    P, batch = _setup(cfg, bs, size, labeled)
    alpha = float(cfg.CONSISTENCY_TRAINER.LOSS_FACTOR)
    outs, loss, grads, sd, seen, math, _ = _gpu_step(cfg, P, batch, dev, monkeypatch)
    assert math == 'bf16'
    _check_routing(seen, 'bf16')
    ref32, loss32, g32, _ = _oracle_step(cfg, P, batch, torch.float32, alpha)
    with bf16_conv_oracle():
        ref16, loss16, g16, _ = _oracle_step(cfg, P, batch, torch.float32, alpha)
    for i, (o, r32, r16) in enumerate(zip(outs, ref32, ref16)):
        e32, e16 = rel(o, r32), rel(o, r16)
        print(f'output {i}: rel err vs fp32 oracle {e32:.2e}, vs bf16-emulating oracle {e16:.2e}')
        assert e32 < 3e-2
        assert e16 < e32
    print(f'loss {loss:.6f} fp32 oracle {loss32:.6f} emulated {loss16:.6f}')
    assert abs(loss - loss32) < 1e-2
    cos = lambda a, b: float(torch.dot(a.double().flatten(), b.double().flatten())
                             / (a.double().norm() * b.double().norm()).clamp_min(1e-30))
    worst, bad = (None, 1.0, 1.0), []
    for k, r in g32.items():
        if k.endswith('conv.0.bias') or k.endswith('conv.3.bias'):
            continue
        c, c16 = cos(grads[k], r), cos(g16[k], r)
        if c < worst[1]:
            worst = (k, c, c16)
        if not (c > 0.85 and c >= c16 - 0.05):
            bad.append((k, c, c16))
    print(f'worst gradient cosine similarity to the fp32 oracle {worst[1]:.4f} (bf16-emulating oracle {worst[2]:.4f}, '
          f'{worst[0]})')
    assert not bad, bad


@pytest.mark.parametrize('config,math', [('baseline_siamese', 'h2'), ('baseline_dualstream', 'bf16'),
                                         ('dtsiamese', 'h2'), ('siamese_mmcr_alpha0500', 'bf16'), ('debug', 'h2')])
def test_create_network_carries_the_config_arithmetic(dev, monkeypatch, config, math):
    """A model built only through create_network(load_cfg(config)) runs the config's arithmetic, launch by launch
    (scd_igemm_arith / scd_wgrad_arith), whatever the process default is."""
    from multimodal_siamese_cd_amd import hip, trainers
    from multimodal_siamese_cd_amd.utils import datasets, experiment_manager as em, networks
    cfg = em.load_cfg(config)
    prev = hip.set_conv_math('f32')  # a different process default must not leak into the model
    try:
        net = networks.create_network(cfg).to(dev).train()
        assert net.module.conv_math == math
        gen = torch.Generator(device=dev).manual_seed(3)
        b = datasets.synthetic_batch(cfg, 2, dev, gen, 64)
        seen = record_arith(monkeypatch, dev)
        trainers.step_loss(cfg, net(b['x_t1'], b['x_t2']), b).backward()
        monkeypatch.undo()
    finally:
        hip.set_conv_math(prev)
    _check_routing(seen, math)
    assert not any(s[4] == 'f32' for s in seen)


def test_models_of_different_arithmetic_coexist(dev):
    """An h2 model and a bf16 model in one process, interleaved: each keeps its own arithmetic and its results equal
    those of the same model run alone."""
    from multimodal_siamese_cd_amd import trainers
    from multimodal_siamese_cd_amd.utils import datasets, experiment_manager as em, networks
    cfg_a = em.load_cfg('debug')
    cfg_b = em.load_cfg('debug')
    cfg_b.MODEL.PRECISION = 'bf16'
    gen = torch.Generator(device=dev).manual_seed(4)
    b = datasets.synthetic_batch(cfg_a, 2, dev, gen, 64)

    def make(cfg):
        torch.manual_seed(0)
        return networks.create_network(cfg).to(dev).train()

    def run(net, cfg):
        net.zero_grad(set_to_none=True)
        out = net(b['x_t1'], b['x_t2'])
        trainers.step_loss(cfg, out, b).backward()
        return out.detach().clone(), [p.grad.clone() for p in net.parameters()]

    na, nb = make(cfg_a), make(cfg_b)
    alone_a, alone_b = run(na, cfg_a), run(nb, cfg_b)
    na, nb = make(cfg_a), make(cfg_b)
    out_a = na(b['x_t1'], b['x_t2'])
    out_b = nb(b['x_t1'], b['x_t2'])  # forward of b between a's forward and a's backward
    trainers.step_loss(cfg_a, out_a, b).backward()
    trainers.step_loss(cfg_b, out_b, b).backward()
    assert torch.equal(out_a.detach(), alone_a[0]) and torch.equal(out_b.detach(), alone_b[0])
    for p, g in zip(na.parameters(), alone_a[1]):
        assert torch.equal(p.grad, g)
    for p, g in zip(nb.parameters(), alone_b[1]):
        assert torch.equal(p.grad, g)
    assert rel(out_a.detach(), out_b.detach()) > 1e-4  # really two arithmetics


def test_baseline_siamese_bs64_north_star_batch(dev, monkeypatch):
    """The north-star batch (bs=64 per GPU, 256x256, SiameseUNet [64,128,256,512], h2): the Siamese level-0 maps are
    128 x 256^2 x 64 fp32 = 2.15 GB, so the level-0 convs and weight grads run as image chunks below 2 GiB
    (DESIGN 3.1c), and the BatchNorm-derived h2 operand bounds (|gamma| sqrt(n-1) + |beta|, n = 4.2 M) are at their
    loosest.  A full training step on the GPU against
      (1) the fp64 oracle following the GPU forward's own ReLU / MaxPool branches (tests/_parity.py; ~100 GB of host
          memory at this batch): logits within 1e-4 (north_star), change masks bit-exact outside the |logit| < 1e-4
          max band, loss within 1e-5, BatchNorm running statistics within 1e-5, num_batches_tracked exact, and EVERY
          gradient tensor within 1e-3 max-relative -- the chunked level-0 weight grads included;
      (2) the reference's own fp32 arithmetic (the fp32 oracle, forward and backward, its own branches): every gradient
          tensor within 2e-2 rel-L2 (the reference-fixture bar; at kink-ambiguous pixels the two take different
          branches, which moves the level-0 weights, downstream of every such pixel, by up to ~3e-3 max-relative)."""
    from oracle import siamese_oracle as O
    cfg = _cfg('baseline_siamese', 'siameseunet', FULL, PRECISION='fp32')
    bs, size = 64, 256
    assert 2 * bs * size * size * FULL[0] * 4 >= 2 ** 31  # the chunked launch path is the one under test
    P, batch = _setup(cfg, bs, size)
    outs, loss, grads, sd, seen, math, (trace, module) = _gpu_step(cfg, P, batch, dev, monkeypatch)
    assert math == 'h2'
    _check_routing(seen, 'h2')
    for k, g in grads.items():
        assert bool(torch.isfinite(g).all()), k
        if k.endswith('conv.0.bias') or k.endswith('conv.3.bias'):  # a pre-BatchNorm bias: true gradient 0
            assert float(g.abs().max()) < 1e-4 * float(grads[k.replace('.bias', '.weight')].abs().max()), k
    torch.cuda.empty_cache()
    ocfg = _ocfg(cfg)
    # (1) branch-matched fp64
    ref_B = O.fresh_buffers(O.param_shapes('siameseunet', ocfg))
    ref_out, ref_loss, ref_g = branch_matched_reference('siameseunet', P, batch, ocfg, trace, module,
                                                        lambda o, bt: O.step_loss('siameseunet', o, bt, 0.5),
                                                        buffers=ref_B)
    del trace
    logits, ref = outs[0], ref_out.detach()
    e = rel(logits, ref)
    mm = mask_mismatch(logits.numpy(), ref.numpy())
    print(f'bs=64: logits rel err {e:.2e}, mask mismatches outside the band {mm}, loss {loss:.7f} vs '
          f'{ref_loss.item():.7f}')
    assert e < 1e-4
    assert mm == 0
    assert abs(loss - ref_loss.item()) < 1e-5
    worst = 0.0
    for k, v in ref_B.items():
        if k.endswith('running_mean') or k.endswith('running_var'):
            worst = max(worst, rel(sd[k], v))
            assert rel(sd[k], v) < 1e-5, k
        elif k.endswith('num_batches_tracked'):
            assert int(sd[k]) == int(v), k
    print(f'bs=64: BatchNorm running statistics worst rel err {worst:.2e}')
    bad = check_branch_matched(grads, ref_g, list(grads), 1e-3)
    assert not bad, bad
    del ref_out, ref_loss, ref_g
    # (2) the fp32 oracle on its own branches
    Pr = {k: v.detach().clone().requires_grad_(True) for k, v in P.items()}
    out32 = O.forward('siameseunet', Pr, O.fresh_buffers(O.param_shapes('siameseunet', ocfg)), batch['x_t1'],
                      batch['x_t2'], ocfg, True)
    O.step_loss('siameseunet', out32, batch, 0.5).backward()
    del out32
    l2, l0 = {}, {}
    for k, r in Pr.items():
        if k.endswith('conv.0.bias') or k.endswith('conv.3.bias'):  # true gradient 0: checked for being ~0 above
            continue
        l2[k] = float((grads[k].double() - r.grad.double()).norm() / r.grad.double().norm().clamp_min(1e-30))
        if k in ('inc.conv.conv.0.weight', 'inc.conv.conv.3.weight'):
            l0[k] = rel(grads[k], r.grad)
    worst = max(l2.items(), key=lambda kv: kv[1])
    print(f'bs=64 gradients vs the fp32 oracle (own branches): worst rel-L2 {worst[1]:.2e} ({worst[0]}); level-0 '
          f'max-rel {l0}')
    assert worst[1] < 2e-2, worst


def _grad_rel_l2(grads, ref):
    """{name: rel-L2} of every gradient tensor but the pre-BatchNorm conv biases (true gradient 0)."""
    out = {}
    for k, r in ref.items():
        if k.endswith('conv.0.bias') or k.endswith('conv.3.bias'):
            continue
        r = r.detach().double()
        out[k] = float((grads[k].double() - r).norm() / r.norm().clamp_min(1e-30))
    return out


def _cos(a, b):
    a, b = a.double().flatten(), b.double().flatten()
    return float(torch.dot(a, b) / (a.norm() * b.norm()).clamp_min(1e-30))


def test_dtsiamese_bs64_shipped_batch(dev, monkeypatch):
    """dtsiamese at its shipped batch (bs=64, 256x256, [64,128,256,512], h2): the fused dual-task encoder (difference
    and the [t2; t1] semantic skips in one pass) and decoder_sem as one 128-image batch with per-date BatchNorm
    segments (level-0 concat 128 x 256^2 x 128 fp32 = 4.3 GB: chunked convs), forward AND backward.  Against the fp32
    oracle's training step (one oracle pass: forward, loss and backward): all three outputs within 1e-4, change /
    semantic masks bit-exact outside the band, the dual-task loss within 1e-5, BatchNorm running statistics within 1e-5
    (decoder_sem's updated t2 then t1), num_batches_tracked exact, and EVERY gradient tensor within 2e-2 rel-L2 -- the
    fp32 oracle takes its own ReLU / pooling branches, so kink-ambiguous pixels move single weights by up to a few
    1e-3 max-relative (printed); the strict 1e-3 max-relative bar against the branch-matched fp64 oracle is held for
    this model at full shapes in test_fp32_workload_matches_oracle[dtsiamese] (bs=2) and for the north-star batch in
    test_baseline_siamese_bs64_north_star_batch (a branch-matched fp64 dtsiamese step at bs=64 needs ~180 GB of host
    memory and minutes of CPU time)."""
    from oracle import siamese_oracle as O
    cfg = _cfg('dtsiamese', 'dtsiameseunet', FULL, PRECISION='fp32')
    bs, size = 64, 256
    P, batch = _setup(cfg, bs, size)
    outs, loss, grads, sd, seen, math, _ = _gpu_step(cfg, P, batch, dev, monkeypatch, trace_bn=False)
    assert math == 'h2'
    _check_routing(seen, 'h2')
    for k, g in grads.items():
        assert bool(torch.isfinite(g).all()), k
    torch.cuda.empty_cache()
    ref, ref_loss, ref_g, B = _oracle_step(cfg, P, batch, torch.float32)
    for i, (o, r) in enumerate(zip(outs, ref)):
        e = rel(o, r)
        mm = mask_mismatch(o.numpy(), r.numpy())
        print(f'dtsiamese bs=64 output {i}: rel err {e:.2e}, mask mismatches outside the band {mm}')
        assert e < 1e-4
        assert mm == 0
    print(f'dtsiamese bs=64 loss {loss:.7f} vs {ref_loss:.7f}')
    assert abs(loss - ref_loss) < 1e-5
    for k, v in B.items():
        if k.endswith('running_mean') or k.endswith('running_var'):
            assert rel(sd[k], v) < 1e-5, k
        elif k.endswith('num_batches_tracked'):
            assert int(sd[k]) == int(v), k
    l2 = _grad_rel_l2(grads, ref_g)
    worst = max(l2.items(), key=lambda kv: kv[1])
    mr = max(((k, rel(grads[k], ref_g[k])) for k in l2), key=lambda kv: kv[1])
    print(f'dtsiamese bs=64 gradients vs the fp32 oracle: {len(l2)} tensors, worst rel-L2 {worst[1]:.2e} ({worst[0]}), '
          f'worst max-rel {mr[1]:.2e} ({mr[0]})')
    assert worst[1] < 2e-2, worst


def _bf16_shipped(dev, monkeypatch, config, model, size, bs, labeled=None):
    """A bf16 workload at its shipped batch, forward and backward, against the fp32 oracle and the bf16-emulating
    oracle (fp32 accumulation: _parity._ACC16), one training-step pass of each: the bs=2 bars of
    test_bf16_workload_matches_oracle on outputs and loss; every gradient tensor's cosine similarity to the fp32
    oracle's within 0.05 of the emulating oracle's own and > 0.85 wherever the emulating oracle reaches 0.9 (a
    relaxation of the bs=2 rule for tensors bf16 arithmetic itself cannot bring to 0.85 at this batch; listed)."""
    cfg = _cfg(config, model, FULL)
    assert str(cfg.MODEL.PRECISION) == 'bf16'
    P, batch = _setup(cfg, bs, size, labeled)
    alpha = float(cfg.CONSISTENCY_TRAINER.LOSS_FACTOR)
    outs, loss, grads, _, seen, math, _ = _gpu_step(cfg, P, batch, dev, monkeypatch, trace_bn=False)
    assert math == 'bf16'
    _check_routing(seen, 'bf16')
    for k, g in grads.items():
        assert bool(torch.isfinite(g).all()), k
    torch.cuda.empty_cache()
    ref32, loss32, g32, _ = _oracle_step(cfg, P, batch, torch.float32, alpha)
    with bf16_conv_oracle(torch.float32):
        ref16, loss16, g16, _ = _oracle_step(cfg, P, batch, torch.float32, alpha)
    for i, (o, r32, r16) in enumerate(zip(outs, ref32, ref16)):
        e32, e16 = rel(o, r32), rel(o, r16)
        print(f'{config} bs={bs} output {i}: rel err vs fp32 oracle {e32:.2e}, vs bf16-emulating oracle {e16:.2e}')
        assert e32 < 3e-2
        assert e16 < e32
    print(f'{config} bs={bs} loss {loss:.6f} fp32 oracle {loss32:.6f} emulated {loss16:.6f}')
    assert abs(loss - loss32) < 1e-2
    worst, bad, n, below = (None, 1.0, 1.0), [], 0, []
    for k, r in g32.items():
        if k.endswith('conv.0.bias') or k.endswith('conv.3.bias'):
            continue
        n += 1
        c, c16 = _cos(grads[k], r), _cos(g16[k], r)
        if c < worst[1]:
            worst = (k, c, c16)
        # every tensor within 0.05 of what the bf16 arithmetic itself reaches (the emulating oracle); the absolute 0.85
        # bar wherever that arithmetic can reach it (c16 >= 0.9): at bs=64 the ConvTranspose bias gradients of the two
        # largest maps (sums over 64 x 128^2 / 256^2 pixels of a bf16-rounded concat gradient, with cancellation) sit
        # at 0.5-0.67 in the emulating oracle too (profiles/r06_shipped_batch_parity.txt) -- bf16's, not the kernels'
        if c16 < 0.9:
            below.append((k, round(c, 4), round(c16, 4)))
        if not (c >= c16 - 0.05 and (c > 0.85 or c16 < 0.9)):
            bad.append((k, c, c16))
    print(f'{config} bs={bs}: {n} gradient tensors, worst cosine similarity to the fp32 oracle {worst[1]:.4f} '
          f'(bf16-emulating oracle {worst[2]:.4f}, {worst[0]}); tensors the bf16 arithmetic itself keeps below 0.9 '
          f'(cosine, emulated cosine): {below}')
    assert not bad, bad


def test_dualstream_bs64_shipped_batch(dev, monkeypatch):
    """baseline_dualstream at its shipped batch (bs=64, bf16 arithmetic and storage, the fused plain encoders, the
    DMA-ring weight grads and the two-decoder head in one launch), forward and backward: logits within 3e-2 of the fp32
    oracle and closer to the bf16-emulating oracle, loss within 1e-2, every gradient's cosine similarity to the fp32
    oracle's > 0.85 and at most 0.05 below the emulating oracle's own."""
    _bf16_shipped(dev, monkeypatch, 'baseline_dualstream', 'dualstreamunet', 256, 64)


def test_mmcr_shipped_batch(dev, monkeypatch):
    """siamese_mmcr_alpha0500 at its shipped batch (configs/siamese_mmcr_base.yaml TRAINER.BATCH_SIZE 4, 512x512
    WhateverNet, bf16): two labelled and two unlabelled samples, so both the supervised terms and the soft-target
    consistency term (non-detached, train_semisupervised.py:100-108) are live; same bars as the dual-stream test."""
    from multimodal_siamese_cd_amd.utils import experiment_manager as em
    assert int(em.load_cfg('siamese_mmcr_alpha0500').TRAINER.BATCH_SIZE) == 4
    _bf16_shipped(dev, monkeypatch, 'siamese_mmcr_alpha0500', 'whatevernet', 512, 4, [True, False, True, False])
