"""Checkpoint interchange with the reference (utils/networks.py:30-56).

tests/golden/siamese_t8-16_checkpoint3.pt was written by the reference's own save_checkpoint after the 3-step
AdamW trajectory of the siamese_t8-16 fixture (tests/golden/make_golden.py).  It is read with
torch.load(weights_only=True).
"""
import numpy as np
import pytest
import torch

from oracle.golden import GOLDEN_DIR, Fixture, rel_err

CKPT = f'{GOLDEN_DIR}/siamese_t8-16_checkpoint3.pt'


def _cfg(tmp=None):
    fx = Fixture('siamese_t8-16')
    cfg = fx.package_cfg()
    cfg.NAME = 'siamese_t8-16'
    if tmp is not None:
        cfg.PATHS.OUTPUT = str(tmp)
    return fx, cfg


def test_reference_checkpoint_loads(tmp_path):
    """load_checkpoint reads the reference's file: parameters = the fixture's params after 3 AdamW steps,
    BatchNorm buffers = its running statistics, AdamW state and step restored."""
    from multimodal_siamese_cd_amd.utils import networks
    fx, cfg = _cfg(tmp_path)
    net, opt, step = networks.load_checkpoint(3, cfg, 'cpu', net_file=CKPT)
    assert step == 3
    sd = net.state_dict()
    for k, v in fx.prefixed('p3/').items():
        assert np.array_equal(sd['module.' + k].numpy(), v), k
    for k, v in fx.prefixed('r3/').items():
        assert np.array_equal(sd['module.' + k].numpy(), v), k
    st = opt.state_dict()
    assert len(st['state']) == len(fx.params0)
    assert all(float(s['step']) == 3.0 for s in st['state'].values())
    g = st['param_groups'][0]
    assert g['lr'] == fx.meta['lr'] and g['weight_decay'] == 0.01


def test_saved_checkpoint_has_the_reference_format(tmp_path):
    """save_checkpoint writes what the reference's load_checkpoint reads: same top-level keys, the same
    module.-prefixed state_dict keys, shapes and dtypes, and an AdamW state of the same structure."""
    from multimodal_siamese_cd_amd.utils import networks
    ref = torch.load(CKPT, weights_only=True)
    fx, cfg = _cfg(tmp_path)
    net = networks.create_network(cfg)
    opt = torch.optim.AdamW(net.parameters(), lr=cfg.TRAINER.LR, weight_decay=0.01)
    for p in net.parameters():  # one optimizer step on CPU to populate the AdamW state
        p.grad = torch.ones_like(p)
    opt.step()
    networks.save_checkpoint(net, opt, 1, 1, cfg)
    ours = torch.load(tmp_path / 'networks' / 'siamese_t8-16_checkpoint1.pt', weights_only=True)
    assert set(ours) == set(ref) == {'step', 'network', 'optimizer'}
    assert list(ours['network']) == list(ref['network'])
    for k, v in ref['network'].items():
        assert ours['network'][k].shape == v.shape and ours['network'][k].dtype == v.dtype, k
    assert set(ours['optimizer']) == set(ref['optimizer'])
    assert list(ours['optimizer']['state']) == list(ref['optimizer']['state'])
    for i, s in ref['optimizer']['state'].items():
        assert set(ours['optimizer']['state'][i]) == set(s)
        for k in ('exp_avg', 'exp_avg_sq'):
            assert ours['optimizer']['state'][i][k].shape == s[k].shape
    rg, og = ref['optimizer']['param_groups'][0], ours['optimizer']['param_groups'][0]
    for k in ('lr', 'betas', 'eps', 'weight_decay', 'amsgrad', 'params'):
        assert og[k] == rg[k], k


@pytest.mark.gpu
def test_reference_checkpoint_resumes_on_gpu():
    """The reference's checkpoint loaded onto the MI355X: train- and eval-mode outputs equal the oracle's at the
    checkpoint's parameters and running statistics, and a further AdamW step runs."""
    from multimodal_siamese_cd_amd import hip, trainers
    from multimodal_siamese_cd_amd.utils import networks
    from oracle import siamese_oracle as O
    hip.load_library()
    dev = torch.device('cuda:0')
    fx, cfg = _cfg()
    net, opt, step = networks.load_checkpoint(3, cfg, dev, net_file=CKPT)
    P = {k: torch.from_numpy(v.copy()) for k, v in fx.prefixed('p3/').items()}
    B = {k: torch.from_numpy(v.copy()) for k, v in fx.prefixed('r3/').items()}
    batch = fx.batch()
    with torch.no_grad():
        ref_eval = O.forward(fx.model_type, P, B, batch['x_t1'], batch['x_t2'], fx.cfg, training=False)
        ref_train = O.forward(fx.model_type, P, dict(B), batch['x_t1'], batch['x_t2'], fx.cfg, training=True)
    net.eval()
    with torch.no_grad():
        ev = net(batch['x_t1'].to(dev), batch['x_t2'].to(dev))
    assert rel_err(ev.cpu().numpy(), ref_eval.numpy()) < 1e-4
    net.train()
    bd = {k: v.to(dev) for k, v in batch.items()}
    out = net(bd['x_t1'], bd['x_t2'])
    assert rel_err(out.detach().cpu().numpy(), ref_train.numpy()) < 1e-4
    loss = trainers.step_loss(cfg, out, bd)
    ref_loss = O.step_loss(fx.model_type, ref_train, batch, fx.meta['alpha'])
    assert abs(loss.item() - ref_loss.item()) < 1e-5
    opt.zero_grad()
    loss.backward()
    opt.step()
    assert all(float(s['step']) == 4.0 for s in opt.state_dict()['state'].values())
