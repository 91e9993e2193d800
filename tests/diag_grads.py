"""Diagnostic (not collected by pytest): per-stage forward values and gradients, HIP path vs CPU oracle.

    python tests/diag_grads.py [fixture]
"""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from multimodal_siamese_cd_amd import engine, hip  # noqa: E402
from multimodal_siamese_cd_amd.utils import networks  # noqa: E402
from oracle import siamese_oracle as O  # noqa: E402
from oracle.golden import Fixture, rel_err  # noqa: E402


def main(name='siamese_t8-16'):
    dev = torch.device('cuda:0')
    hip.load_library()
    fx = Fixture(name)
    cfg = fx.package_cfg()
    net = networks.create_network(cfg)
    with torch.no_grad():
        for k, p in net.module.named_parameters():
            p.copy_(torch.from_numpy(fx.params0[k]))
    m = net.module.to(dev).train()
    batch = fx.batch()
    xb = {k: v.to(dev) for k, v in batch.items()}
    x = engine.pack_pair(xb['x_t1'], xb['x_t2'])
    feats = engine.run_encoder(m.inc, m.encoder, x, 2, True)
    for f in feats:
        f.retain_grad()
    diffs = [engine.siamese_diff(f) for f in feats]
    for d in diffs:
        d.retain_grad()
    dec = engine.run_decoder(m.decoder, diffs[::-1], True)
    dec.retain_grad()
    logits = engine.run_head(m.outc, dec)
    loss = engine.power_jaccard(logits, xb['y_change'])
    loss.backward()

    # oracle with retained intermediates
    P = {k: torch.from_numpy(v.copy()).requires_grad_(True) for k, v in fx.params0.items()}
    B = O.fresh_buffers(O.param_shapes(fx.model_type, fx.cfg))
    topo = fx.cfg['TOPOLOGY']
    f1 = O.encoder(batch['x_t1'], P, B, 'inc.', 'encoder.', topo, True)[::-1]
    f2 = O.encoder(batch['x_t2'], P, B, 'inc.', 'encoder.', topo, True)[::-1]
    for t in f1 + f2:
        t.retain_grad()
    od = O.diff(f1, f2)
    for t in od:
        t.retain_grad()
    odec = O.decoder(od[::-1], P, B, 'decoder.', topo, True)
    odec.retain_grad()
    ologits = O.out_conv(odec, P, 'outc.')
    oloss = O.power_jaccard_loss(ologits, batch['y_change'])
    oloss.backward()

    def nhwc(t):
        return t.permute(0, 2, 3, 1).detach().numpy()

    b = batch['x_t1'].shape[0]
    print(f'loss hip {loss.item():.7f} oracle {oloss.item():.7f}')
    print(f'logits rel {rel_err(logits.detach().cpu().numpy(), ologits.detach().numpy()):.2e}')
    print(f'dec     rel {rel_err(dec.detach().cpu().numpy(), nhwc(odec)):.2e}  grad {rel_err(dec.grad.cpu().numpy(), nhwc(odec.grad)):.2e}')
    for lvl in range(len(feats)):
        fh = feats[lvl].detach().cpu().numpy()
        fo = np.concatenate([nhwc(f1[lvl]), nhwc(f2[lvl])])
        gh = feats[lvl].grad.cpu().numpy()
        go = np.concatenate([nhwc(f1[lvl].grad), nhwc(f2[lvl].grad)])
        dg = diffs[lvl].grad.cpu().numpy()
        dgo = nhwc(od[lvl].grad)
        print(f'level {lvl}: feat rel {rel_err(fh, fo):.2e}  diff-grad rel {rel_err(dg, dgo):.2e}  '
              f'feat-grad rel {rel_err(gh, go):.2e}  shape {fh.shape}')
    for k, p in m.named_parameters():
        if p.grad is None or k.endswith('conv.0.bias') or k.endswith('conv.3.bias'):
            continue
        e = rel_err(p.grad.cpu().numpy(), P[k].grad.numpy())
        flag = '  <<<' if e > 1e-4 else ''
        print(f'{k:55s} {e:.2e}{flag}')


if __name__ == '__main__':
    main(*sys.argv[1:])
