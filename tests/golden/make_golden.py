"""Generate golden fixtures by running the REFERENCE implementation itself (build container only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py  [--ref /root/reference]

Imports the reference's utils/networks.py and utils/loss_functions.py from /root/reference (a local
stub stands in for the missing `fvcore` package, which networks.py only uses for type annotations via
utils/experiment_manager.py:7), builds each model with `networks.create_network` (networks.py:12-27),
loads a deterministic parameter fill (oracle.siamese_oracle.deterministic_params), and records on CPU
fp32 one training step of the reference trainers:

  train-mode outputs, loss, every parameter gradient, BatchNorm buffers after the step,
  eval-mode outputs (running statistics), then two more AdamW steps (loss trajectory + final params).

Only data (inputs and expected outputs) is written to tests/golden/*.npz; no reference source travels.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import siamese_oracle as O  # noqa: E402

CONFIGS = [
    # name, model type, topology, in_channels, S1 bands, S2 bands, batch, hw, labeled
    ('siamese_t8-16', 'siameseunet', [8, 16], 5, [0, 1], [2, 1, 0], 2, 64, None),
    ('siamese_t8-16-32', 'siameseunet', [8, 16, 32], 5, [0, 1], [2, 1, 0], 2, 32, None),
    ('unet_t8-16', 'unet', [8, 16], 5, [0, 1], [2, 1, 0], 2, 32, None),
    ('dualstream_t8-16', 'dualstreamunet', [8, 16], 5, [0, 1], [2, 1, 0], 2, 32, None),
    ('dtsiamese_t8-16', 'dtsiameseunet', [8, 16], 5, [0, 1], [2, 1, 0], 2, 32, None),
    ('whatevernet_t8-16', 'whatevernet', [8, 16], 5, [0, 1], [2, 1, 0], 2, 32, [True, False]),
    # tiles not divisible by 2**levels: MaxPool floors and Up zero-pads the upsampled map (networks.py:437-443)
    ('siamese_t8-16-32_odd', 'siameseunet', [8, 16, 32], 5, [0, 1], [2, 1, 0], 2, (37, 45), None),
    ('dualstream_t8-16_odd', 'dualstreamunet', [8, 16], 5, [0, 1], [2, 1, 0], 1, (27, 30), None),
    ('whatevernet2_t8-16', 'whatevernet2', [8, 16], 5, [0, 1], [2, 1, 0], 2, 32, [True, False]),
    # channel counts that take the production kernels (16x16x32 halo / h2 paths: source channels multiple of 32)
    ('siamese_t32-64', 'siameseunet', [32, 64], 5, [0, 1], [2, 1, 0], 2, 64, None),
    ('dtsiamese_t32-64', 'dtsiameseunet', [32, 64], 5, [0, 1], [2, 1, 0], 2, 64, None),
    ('dualstream_t32-64', 'dualstreamunet', [32, 64], 5, [0, 1], [2, 1, 0], 2, 64, None),
    # channel counts off the kernels' granule of 8 (the twin padding of utils/networks.py); [6, 12] puts two 6-wide
    # halves into the Up and head concats (12 -> 2 x 8, not a 16-wide prefix)
    ('siamese_t12-20', 'siameseunet', [12, 20], 5, [0, 1], [2, 1, 0], 2, 32, None),
    ('dualstream_t6-12', 'dualstreamunet', [6, 12], 5, [0, 1], [2, 1, 0], 2, 32, None),
]
LR = 1e-3
WD = 0.01
ALPHA = 0.5
SEED = 7


def import_reference(ref):
    fv = types.ModuleType('fvcore')
    fvc = types.ModuleType('fvcore.common')
    fvcc = types.ModuleType('fvcore.common.config')

    class _CfgNode(dict):  # annotation-only stand-in
        pass

    fvcc.CfgNode = _CfgNode
    sys.modules.setdefault('fvcore', fv)
    sys.modules.setdefault('fvcore.common', fvc)
    sys.modules.setdefault('fvcore.common.config', fvcc)
    sys.path.insert(0, ref)
    from utils import loss_functions, networks  # noqa: E402
    return networks, loss_functions


def ns_cfg(d):
    from types import SimpleNamespace as NS
    return NS(MODEL=NS(TYPE=d['TYPE'], IN_CHANNELS=d['IN_CHANNELS'], OUT_CHANNELS=d['OUT_CHANNELS'],
                       TOPOLOGY=list(d['TOPOLOGY'])),
              DATALOADER=NS(S1_BANDS=list(d['S1_BANDS']), S2_BANDS=list(d['S2_BANDS'])))


def outputs_list(o):
    return list(o) if isinstance(o, (tuple, list)) else [o]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--ref', default='/root/reference')
    ap.add_argument('--only', default=None)
    args = ap.parse_args()
    networks, loss_functions = import_reference(args.ref)
    if args.only in (None, 'metrics'):
        make_metrics_fixture()
        if args.only == 'metrics':
            return
    pj = loss_functions.get_criterion('PowerJaccardLoss')
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    if args.only in (None, DP_NAME):
        make_dataparallel_fixture(networks, pj)
        if args.only == DP_NAME:
            return

    for name, mtype, topo, cin, s1, s2, b, hw, labeled in CONFIGS:
        if args.only and args.only != name:
            continue
        cfgd = dict(TYPE=mtype, IN_CHANNELS=cin, OUT_CHANNELS=1, TOPOLOGY=topo, S1_BANDS=s1, S2_BANDS=s2)
        net = networks.create_network(ns_cfg(cfgd))
        module = net.module
        shapes = O.param_shapes(mtype, cfgd)
        ref_shapes = [(k, tuple(p.shape)) for k, p in module.named_parameters()]
        assert ref_shapes == list(shapes.items()), f'{name}: oracle parameter table differs from the reference'
        P0 = O.deterministic_params(shapes, SEED)
        with torch.no_grad():
            for k, p in module.named_parameters():
                p.copy_(P0[k])
        batch = O.synthetic_batch(cfgd, b, hw, SEED + 1, labeled)
        rec = {}
        for k in ('x_t1', 'x_t2', 'y_change', 'y_sem_t1', 'y_sem_t2'):
            rec[k] = batch[k].numpy()
        rec['is_labeled'] = batch['is_labeled'].numpy()
        for k, v in P0.items():
            rec['p0/' + k] = v.numpy()

        opt = torch.optim.AdamW(net.parameters(), lr=LR, weight_decay=WD)
        net.train()
        opt.zero_grad()
        out = net(batch['x_t1'], batch['x_t2'])
        # the loss recipes of the reference trainers, evaluated with the REFERENCE loss function
        loss = _ref_step_loss(mtype, out, batch, pj)
        loss.backward()
        for i, o in enumerate(outputs_list(out)):
            rec[f'out/{i}'] = o.detach().numpy()
        rec['loss0'] = np.float32(loss.item())
        for k, p in module.named_parameters():
            if p.grad is not None:  # outc_sem_change is unused by DualTaskSiameseUNet.forward
                rec['g/' + k] = p.grad.detach().numpy().copy()
        for k, v in module.state_dict().items():
            if 'running' in k or 'num_batches' in k:
                rec['r1/' + k] = v.detach().numpy().copy()
        net.eval()
        with torch.no_grad():
            ev = net(batch['x_t1'], batch['x_t2'])
        for i, o in enumerate(outputs_list(ev)):
            rec[f'eval/{i}'] = o.numpy()
        net.train()
        losses = [loss.item()]
        opt.step()
        for _ in range(2):
            opt.zero_grad()
            out = net(batch['x_t1'], batch['x_t2'])
            loss = _ref_step_loss(mtype, out, batch, pj)
            loss.backward()
            opt.step()
            losses.append(loss.item())
        rec['losses'] = np.array(losses, dtype=np.float32)
        if name == 'siamese_t8-16':
            save_reference_checkpoint(networks, net, opt, ns_cfg(cfgd), name)
        for k, p in module.named_parameters():
            rec['p3/' + k] = p.detach().numpy().copy()
        for k, v in module.state_dict().items():
            if 'running' in k or 'num_batches' in k:
                rec['r3/' + k] = v.detach().numpy().copy()
        meta = dict(name=name, cfg=cfgd, batch=b, hw=hw, seed=SEED, lr=LR, wd=WD, alpha=ALPHA, labeled=labeled,
                    generator='reference utils/networks.py + utils/loss_functions.py (CPU fp32, torch '
                              + torch.__version__ + ')')
        rec['meta'] = np.array(json.dumps(meta))
        path = os.path.join(HERE, f'{name}.npz')
        np.savez_compressed(path, **rec)
        print(f'{name}: loss0={losses[0]:.6f} losses={losses} -> {os.path.getsize(path) / 1024:.0f} KiB')


DP_NAME = 'siamese_t8-16_dp2'


def make_dataparallel_fixture(networks, pj, shards=2, per_shard=2, hw=32):
    """nn.DataParallel's computation on `shards` devices (utils/networks.py:27, train_supervised.py:71-76), run with
    the reference modules on the CPU: the batch is scattered along dim 0, every replica runs its shard with its own
    BatchNorm batch statistics, the logits are gathered and ONE power_jaccard_loss is taken over the gathered batch;
    the replicas' parameter gradients are reduce-added (here: one module called per shard, so autograd sums them);
    running statistics persist from replica 0 only (torch/nn/parallel/data_parallel.py: the device-0 replica shares
    the module's buffers), so the other shards' buffer updates are undone."""
    name = DP_NAME
    cfgd = dict(TYPE='siameseunet', IN_CHANNELS=5, OUT_CHANNELS=1, TOPOLOGY=[8, 16], S1_BANDS=[0, 1], S2_BANDS=[2, 1, 0])
    net = networks.create_network(ns_cfg(cfgd))
    module = net.module
    P0 = O.deterministic_params(O.param_shapes('siameseunet', cfgd), SEED)
    with torch.no_grad():
        for k, p in module.named_parameters():
            p.copy_(P0[k])
    batch = O.synthetic_batch(cfgd, shards * per_shard, hw, SEED + 3)
    rec = {k: batch[k].numpy() for k in ('x_t1', 'x_t2', 'y_change', 'y_sem_t1', 'y_sem_t2')}
    rec['is_labeled'] = batch['is_labeled'].numpy()
    for k, v in P0.items():
        rec['p0/' + k] = v.numpy()
    module.train()
    outs = []
    params = dict(module.named_parameters())
    for sh in range(shards):
        sl = slice(sh * per_shard, (sh + 1) * per_shard)
        if sh == 0:  # replica 0: the module itself (its buffers take the running-statistics update)
            outs.append(module(batch['x_t1'][sl], batch['x_t2'][sl]))
        else:  # another replica: the same parameters, private copies of the buffers (discarded)
            bufs = {k: v.clone() for k, v in module.named_buffers()}
            outs.append(torch.func.functional_call(module, {**params, **bufs}, (batch['x_t1'][sl], batch['x_t2'][sl])))
    logits = torch.cat(outs, 0)
    loss = pj(logits, batch['y_change'])
    loss.backward()
    rec['out/0'] = logits.detach().numpy()
    rec['loss0'] = np.float32(loss.item())
    for k, p in module.named_parameters():
        rec['g/' + k] = p.grad.detach().numpy().copy()
    for k, v in module.state_dict().items():
        if 'running' in k or 'num_batches' in k:
            rec['r1/' + k] = v.detach().numpy().copy()
    meta = dict(name=name, cfg=cfgd, batch=shards * per_shard, shards=shards, hw=hw, seed=SEED, lr=LR, wd=WD,
                alpha=ALPHA, labeled=None,
                generator='reference utils/networks.py + utils/loss_functions.py run per shard as nn.DataParallel '
                          '(CPU fp32, torch ' + torch.__version__ + ')')
    rec['meta'] = np.array(json.dumps(meta))
    path = os.path.join(HERE, f'{name}.npz')
    np.savez_compressed(path, **rec)
    print(f'{name}: loss0={loss.item():.6f} -> {os.path.getsize(path) / 1024:.0f} KiB')


def make_metrics_fixture():
    """utils/metrics.py MultiThresholdMetric (metrics.py:5-59) over three add_sample calls.

    Probabilities include exact threshold values, their fp32 neighbours, 0, 1 and NaN, so the
    round(p - t + 0.5) decision (metrics.py:26) is pinned at its ties; one label is NaN (bool() -> True)."""
    from utils import metrics
    rng = np.random.default_rng(SEED + 100)
    thr = torch.linspace(0, 1, 11)
    m = metrics.MultiThresholdMetric(thr)
    m5 = metrics.MultiThresholdMetric(torch.linspace(0.5, 1, 1))  # utils/evaluation.py:12
    rec = {'thresholds': thr.numpy()}
    for i, (b, h, w) in enumerate([(2, 16, 24), (1, 37, 45), (3, 8, 8)]):
        p = rng.random((b, 1, h, w), dtype=np.float32)
        flat = p.reshape(-1)
        ties = np.concatenate([thr.numpy(), np.nextafter(thr.numpy(), 2), np.nextafter(thr.numpy(), -1),
                               np.float32([0, 1, 0.5, np.nan])]).astype(np.float32)
        flat[:ties.size] = np.clip(ties, 0, 1) if i else ties
        y = (rng.random((b, 1, h, w)) > 0.6).astype(np.float32)
        if i == 0:
            y.reshape(-1)[-1] = np.nan
        rec[f'y_pred/{i}'] = p
        rec[f'y_true/{i}'] = y
        m.add_sample(torch.from_numpy(y), torch.from_numpy(p))
        m5.add_sample(torch.from_numpy(y), torch.from_numpy(p))
    for k in ('TP', 'TN', 'FP', 'FN'):
        rec[k] = getattr(m, k).numpy()
        rec['eval_' + k] = getattr(m5, k).numpy()
    rec['precision'] = m.precision.numpy()
    rec['recall'] = m.recall.numpy()
    rec['f1'] = m.compute_f1().numpy()
    fpr, fnr = m.compute_basic_metrics()
    rec['fpr'] = fpr.numpy()
    rec['fnr'] = fnr.numpy()
    rec['eval_f1'] = m5.compute_f1().numpy()
    rec['meta'] = np.array(json.dumps(dict(name='metrics', generator='reference utils/metrics.py (CPU, torch '
                                           + torch.__version__ + ')')))
    path = os.path.join(HERE, 'metrics_mt.npz')
    np.savez_compressed(path, **rec)
    print(f'metrics: f1={rec["f1"]} -> {os.path.getsize(path) / 1024:.0f} KiB')


def save_reference_checkpoint(networks, net, opt, cfg, name):
    """The reference's own save_checkpoint (utils/networks.py:30-38) after the 3-step trajectory: a checkpoint
    file in the reference's format ({'step', 'network' (module.-prefixed), 'optimizer' (AdamW state)})."""
    import shutil
    import tempfile
    from types import SimpleNamespace as NS
    tmp = tempfile.mkdtemp()
    cfg.PATHS = NS(OUTPUT=tmp)
    cfg.NAME = name
    os.makedirs(os.path.join(tmp, 'networks'), exist_ok=True)
    networks.save_checkpoint(net, opt, 3, 3, cfg)
    dst = os.path.join(HERE, f'{name}_checkpoint3.pt')
    shutil.copy(os.path.join(tmp, 'networks', f'{name}_checkpoint3.pt'), dst)
    shutil.rmtree(tmp)
    print(f'{name}: reference checkpoint -> {os.path.getsize(dst) / 1024:.0f} KiB')


def _ref_step_loss(mtype, out, batch, pj):
    """Loss recipes of train_supervised.py:75, train_supervised_dualtask.py:73-85, train_semisupervised.py:82-113."""
    y = batch['y_change']
    if mtype in ('siameseunet', 'unet', 'dualstreamunet'):
        return pj(out, y)
    if mtype == 'dtsiameseunet':
        c, s1, s2 = out
        return (pj(c, y) + (pj(s1, batch['y_sem_t1']) + pj(s2, batch['y_sem_t2'])) / 2) / 2
    if mtype in ('whatevernet', 'whatevernet2'):
        f, s1, s2 = out
        lab = batch['is_labeled']
        loss = None
        if lab.any():
            loss = ALPHA * ((pj(f[lab], y[lab]) + pj(s1[lab], y[lab]) + pj(s2[lab], y[lab])) / 3)
        if not lab.all():
            nl = torch.logical_not(lab)
            cons = (1 - ALPHA) * pj(s1[nl], torch.sigmoid(s2[nl]))
            loss = cons if loss is None else loss + cons
        return loss
    raise ValueError(mtype)


if __name__ == '__main__':
    main()
