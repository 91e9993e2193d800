"""Exact-DataParallel mode on the HIP path (MI355X): two ranks on one GPU (gloo carries the collectives of the
rehearsal; on a node the same code runs over RCCL) against the reference's own nn.DataParallel computation
(tests/golden/siamese_t8-16_dp2.npz: the reference modules run per shard, one power_jaccard_loss over the gathered
logits, replica gradients reduce-added, replica-0 running statistics).

The loss kernels' partial sums are SUM-all-reduced before the loss is formed (scd_pjaccard_loss_from_sums) and the
gradient buckets are summed (parallel.sum_allreduce_hook).  Bars as tests/test_model_gpu.py: logits 1e-4, loss
1e-5, gradients 1e-3 (tests/_parity.py kink rule), running statistics 1e-5.
"""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR='127.0.0.1',
                      MASTER_PORT=str(port), SCD_RANKS_SHARE_GPU='1')
    from multimodal_siamese_cd_amd import hip, parallel, trainers
    from multimodal_siamese_cd_amd.utils import networks
    from oracle.golden import Fixture
    parallel.init_distributed('gloo')
    dev = torch.device('cuda', parallel.device_index(rank))
    torch.cuda.set_device(dev)
    hip.load_library()
    fx = Fixture('siamese_t8-16_dp2')
    cfg = fx.package_cfg()
    net = networks.create_network(cfg)
    with torch.no_grad():
        for k, p in net.module.named_parameters():
            p.copy_(torch.from_numpy(fx.params0[k]))
    net = parallel.wrap_ddp(net.to(dev), dev, exact_dataparallel=True).train()
    per = fx.meta['batch'] // world
    b = {k: v[rank * per:(rank + 1) * per].to(dev) for k, v in fx.batch().items()}
    out = net(b['x_t1'], b['x_t2'])
    loss = trainers.step_loss(cfg, out, b, net)
    loss.backward()
    torch.cuda.synchronize()
    torch.save({'loss': loss.item(), 'logits': out.detach().cpu(),
                'grads': {n: p.grad.detach().cpu() for n, p in net.module.named_parameters()},
                'buffers': {n: v.detach().cpu() for n, v in net.module.named_buffers()}},
               os.path.join(out_dir, f'rank{rank}.pt'))
    torch.distributed.destroy_process_group()


@pytest.mark.timeout(300)
def test_exact_dataparallel_two_ranks_match_reference():
    from _parity import check_gradients, record_kinks
    from oracle import siamese_oracle as O
    from oracle.golden import Fixture, rel_err
    fx = Fixture('siamese_t8-16_dp2')
    world = fx.meta['shards']
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), d), nprocs=world, join=True)
        res = [torch.load(os.path.join(d, f'rank{r}.pt'), weights_only=True) for r in range(world)]
    logits = np.concatenate([r['logits'].numpy() for r in res])
    assert rel_err(logits, fx.outputs[0]) < 1e-4
    for r in res:
        assert abs(r['loss'] - float(fx.z['loss0'])) < 1e-5
    # kink-ambiguous pre-activations of either shard's forward (BatchNorm statistics are per shard)
    per = fx.meta['batch'] // world
    P = {k: torch.from_numpy(v.copy()) for k, v in fx.params0.items()}
    full = fx.batch()
    kinks = []
    for s in range(world):
        bs = {k: v[s * per:(s + 1) * per] for k, v in full.items()}
        kinks += record_kinks('siameseunet', P, O.fresh_buffers(O.param_shapes('siameseunet', fx.cfg)), bs, fx.cfg,
                              torch.float32, 1e-6)
    ref = {k: torch.from_numpy(v) for k, v in fx.grads.items()}
    order = list(res[0]['grads'])
    for r in res:
        assert not check_gradients(r['grads'], ref, order, {k: 1e-3 for k in order}, kinks)
    for n, v in fx.prefixed('r1/').items():
        got = res[0]['buffers'][n].numpy()
        if n.endswith('num_batches_tracked'):
            assert int(got) == int(v), n
        else:
            assert rel_err(got, v) < 1e-5, n


def test_loss_from_global_sums_kernel(dev=None):
    """scd_pjaccard_loss_from_sums / scd_jaccard_multi_loss_from_sums: the sums of two shards added and re-formed give
    the loss of the concatenated batch, and the backward with those global sums gives each shard's slice of the
    concatenated batch's gradient."""
    from multimodal_siamese_cd_amd import hip
    hip.load_library()
    dev = torch.device('cuda:0')
    g = torch.Generator().manual_seed(2)
    z = torch.randn(4, 1, 33, 40, generator=g).to(dev)
    t = (torch.rand(4, 1, 33, 40, generator=g) > 0.8).float().to(dev)
    ws = torch.empty(hip.pjaccard_workspace_bytes(z.numel()), dtype=torch.uint8, device=dev)
    s_all, l_all = torch.empty(3, device=dev), torch.empty((), device=dev)
    hip.pjaccard_fwd(z, t, s_all, l_all, ws)
    parts = []
    for sl in (slice(0, 2), slice(2, 4)):
        s, l_ = torch.empty(3, device=dev), torch.empty((), device=dev)
        hip.pjaccard_fwd(z[sl].contiguous(), t[sl].contiguous(), s, l_, ws)
        parts.append(s)
    glob = parts[0] + parts[1]
    loss = torch.empty((), device=dev)
    hip.pjaccard_loss_from_sums(glob, loss)
    assert abs(loss.item() - l_all.item()) < 1e-6
    assert abs(glob[2].item() - s_all[2].item()) <= 1e-6 * s_all[2].item()
    gz_all = torch.empty_like(z)
    hip.pjaccard_bwd(z, t, s_all, None, gz_all)
    gz0 = torch.empty_like(z[:2])
    hip.pjaccard_bwd(z[:2].contiguous(), t[:2].contiguous(), glob, None, gz0)
    assert ((gz0 - gz_all[:2]).abs().max() / gz_all.abs().max()).item() < 1e-5
    # multi-term form: a labelled and an unlabelled sample per shard, the MMCR consistency term among the terms
    lab = torch.tensor([1, 0, 1, 0], dtype=torch.uint8, device=dev)
    z2 = torch.randn(4, 1, 33, 40, generator=g).to(dev)
    terms = lambda zz, tt, zz2: [dict(logits=zz, target=tt, coef=0.25, select=1, soft=0),
                                 dict(logits=zz, target=zz2, coef=0.5, select=2, soft=1)]
    sums_all, loss_all = torch.empty((2, 4), device=dev), torch.empty((), device=dev)
    hip.jaccard_multi_fwd(terms(z, t, z2), lab, 4, 33 * 40, sums_all, loss_all)
    acc = torch.zeros((2, 4), device=dev)
    for sl in (slice(0, 2), slice(2, 4)):
        sm, lm = torch.empty((2, 4), device=dev), torch.empty((), device=dev)
        hip.jaccard_multi_fwd(terms(z[sl].contiguous(), t[sl].contiguous(), z2[sl].contiguous()), lab[sl].contiguous(),
                              2, 33 * 40, sm, lm)
        acc += sm
    lm = torch.empty((), device=dev)
    hip.jaccard_multi_loss_from_sums(terms(z, t, z2), acc, lm)
    assert abs(lm.item() - loss_all.item()) < 1e-6
    assert torch.equal(acc[:, 3], sums_all[:, 3])


# ---------------------------------------------------------------------------------------------------------------------
# The variant models of the configs that scale (baseline_dualstream, dtsiamese): 2 ranks in exact-DataParallel mode
# against ONE process computing nn.DataParallel's function on the same GPU -- each shard's forward separately (per-shard
# BatchNorm statistics, utils/networks.py:27), one loss over the concatenated outputs, the shards' gradients summed by
# autograd.  Both sides run the same kernels on the same per-shard shapes, so outputs are bit-identical per shard; the
# loss partial sums are reduced in a different order (all-reduce of per-shard sums vs one pass), so loss and
# gradients agree to 1e-5.
# ---------------------------------------------------------------------------------------------------------------------
_VARIANTS = {
    # id: (config, model, topology, tile, batch per rank)
    'dualstream': ('baseline_dualstream', 'dualstreamunet', [64, 128], 64, 2),
    'dtsiamese': ('dtsiamese', 'dtsiameseunet', [64, 128], 64, 2),
}


def _variant_setup(vid, world):
    from multimodal_siamese_cd_amd.utils import experiment_manager as em
    from oracle import siamese_oracle as O
    config, model, topo, size, per = _VARIANTS[vid]
    cfg = em.load_cfg(config)
    cfg.MODEL.TYPE, cfg.MODEL.TOPOLOGY = model, list(topo)
    ocfg = dict(TYPE=model, TOPOLOGY=list(topo), IN_CHANNELS=cfg.MODEL.IN_CHANNELS,
                OUT_CHANNELS=cfg.MODEL.OUT_CHANNELS, S1_BANDS=list(cfg.DATALOADER.S1_BANDS),
                S2_BANDS=list(cfg.DATALOADER.S2_BANDS))
    P = O.deterministic_params(O.param_shapes(model, ocfg), 11)
    batch = O.synthetic_batch(ocfg, per * world, size, 12)
    return cfg, P, batch, per


def _variant_net(cfg, P, dev):
    from multimodal_siamese_cd_amd.utils import networks
    net = networks.create_network(cfg)
    with torch.no_grad():
        for k, p in net.module.named_parameters():
            p.copy_(P[k])
    return net.to(dev).train()


def _outs(o):
    return list(o) if isinstance(o, (tuple, list)) else [o]


def _variant_worker(rank, world, port, out_dir, vid):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR='127.0.0.1',
                      MASTER_PORT=str(port), SCD_RANKS_SHARE_GPU='1')
    from multimodal_siamese_cd_amd import hip, parallel, trainers
    parallel.init_distributed('gloo')
    dev = torch.device('cuda', parallel.device_index(rank))
    torch.cuda.set_device(dev)
    hip.load_library()
    cfg, P, batch, per = _variant_setup(vid, world)
    net = parallel.wrap_ddp(_variant_net(cfg, P, dev), dev, exact_dataparallel=True)
    b = {k: v[rank * per:(rank + 1) * per].to(dev) for k, v in batch.items()}
    out = net(b['x_t1'], b['x_t2'])
    loss = trainers.step_loss(cfg, out, b, net)
    loss.backward()
    torch.cuda.synchronize()
    torch.save({'loss': loss.item(), 'outs': [o.detach().cpu() for o in _outs(out)],
                'grads': {n: p.grad.detach().cpu() for n, p in net.module.named_parameters() if p.grad is not None}},
               os.path.join(out_dir, f'rank{rank}.pt'))
    torch.distributed.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize('vid', list(_VARIANTS))
def test_exact_dataparallel_variants_two_ranks_match_one_process(vid):
    from multimodal_siamese_cd_amd import hip, trainers
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_variant_worker, args=(world, _free_port(), d, vid), nprocs=world, join=True)
        res = [torch.load(os.path.join(d, f'rank{r}.pt'), weights_only=True) for r in range(world)]
    # one process: DataParallel's function (per-shard forwards, one loss over the gathered outputs, summed gradients)
    hip.load_library()
    dev = torch.device('cuda:0')
    cfg, P, batch, per = _variant_setup(vid, world)
    net = _variant_net(cfg, P, dev)
    b = {k: v.to(dev) for k, v in batch.items()}
    shard_outs = [_outs(net(b['x_t1'][s * per:(s + 1) * per], b['x_t2'][s * per:(s + 1) * per]))
                  for s in range(world)]
    outs = [torch.cat([so[i] for so in shard_outs]) for i in range(len(shard_outs[0]))]
    loss = trainers.step_loss(cfg, outs if len(outs) > 1 else outs[0], b)
    loss.backward()
    torch.cuda.synchronize()
    for r, so in zip(res, shard_outs):  # each rank's outputs: the same kernels on the same shard, bit-identical
        for a, e in zip(r['outs'], so):
            assert torch.equal(a, e.detach().cpu())
        assert abs(r['loss'] - loss.item()) <= 1e-5 * abs(loss.item())
    worst = 0.0
    for n, p in net.named_parameters():
        k = n.split('module.', 1)[-1]
        if p.grad is None:  # outside the forward graph (dtsiamese's outc_sem_change, assessment_semantics.py:34)
            assert all(k not in r['grads'] for r in res), k
            continue
        ref = p.grad.detach().cpu().double()
        for r in res:
            e = ((r['grads'][k].double() - ref).abs().max() / ref.abs().max().clamp_min(1e-30)).item()
            worst = max(worst, e)
            assert e < 1e-5 or k.endswith(('conv.0.bias', 'conv.3.bias')), (k, e)
    print(f'{vid}: exact-DataParallel 2 ranks vs one process, worst gradient max-rel {worst:.2e}')
