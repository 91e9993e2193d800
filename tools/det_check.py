"""Run-to-run determinism of the training step: the same AdamW steps repeated in fresh models, compared bitwise
per step (logits, every parameter gradient) against the first run.

    python tools/det_check.py [--runs 3] [--math h2] [--topo 32,64,128,256] [--size 128] [--batch 4]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from multimodal_siamese_cd_amd import hip  # noqa: E402
from multimodal_siamese_cd_amd.utils import experiment_manager, loss_functions, networks  # noqa: E402
from oracle import siamese_oracle as O  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--runs', type=int, default=3)
    ap.add_argument('--math', default='h2')
    ap.add_argument('--topo', default='32,64,128,256')
    ap.add_argument('--size', type=int, default=128)
    ap.add_argument('--batch', type=int, default=4)
    ap.add_argument('--steps', type=int, default=3)
    args = ap.parse_args()
    hip.load_library()
    dev = torch.device('cuda:0')
    topo = [int(t) for t in args.topo.split(',')]
    ocfg = dict(TOPOLOGY=topo, IN_CHANNELS=5, OUT_CHANNELS=1, S1_BANDS=[0, 1], S2_BANDS=[2, 1, 0])
    P = O.deterministic_params(O.param_shapes('siameseunet', ocfg), 7)
    b = {k: v.to(dev) for k, v in O.synthetic_batch(ocfg, args.batch, args.size, 8).items()}
    cfg = experiment_manager.new_config()
    cfg.MODEL.TYPE, cfg.MODEL.IN_CHANNELS, cfg.MODEL.OUT_CHANNELS = 'siameseunet', 5, 1
    cfg.MODEL.TOPOLOGY = topo
    cfg.DATALOADER.S1_BANDS, cfg.DATALOADER.S2_BANDS = [0, 1], [2, 1, 0]
    cfg.MODEL.CONV_MATH = args.math
    crit = loss_functions.get_criterion('PowerJaccardLoss')
    ref = None
    for run in range(args.runs):
        net = networks.create_network(cfg)
        with torch.no_grad():
            for k, p in net.module.named_parameters():
                p.copy_(P[k])
        net.to(dev).train()
        opt = torch.optim.AdamW(net.parameters(), lr=1e-3, weight_decay=0.01)
        rec = []
        for _ in range(args.steps):
            opt.zero_grad(set_to_none=True)
            out = net(b['x_t1'], b['x_t2'])
            loss = crit(out, b['y_change'])
            loss.backward()
            rec.append((out.detach().cpu(), loss.item(),
                        {k: p.grad.detach().cpu().clone() for k, p in net.module.named_parameters()}))
            opt.step()
        if ref is None:
            ref = rec
            print(f'run {run}: reference, losses {[r[1] for r in rec]}', flush=True)
            continue
        bad = []
        for s, ((o, l, g), (o0, l0, g0)) in enumerate(zip(rec, ref)):
            if not torch.equal(o, o0):
                bad.append(f'step {s} logits max|d| {float((o - o0).abs().max()):.3e}')
            for k in g0:
                if not torch.equal(g[k], g0[k]):
                    d = (g[k] - g0[k]).abs()
                    bad.append(f'step {s} {k} {int((d > 0).sum())}/{d.numel()} differ, max|d| {float(d.max()):.3e} '
                               f'(max|g| {float(g0[k].abs().max()):.3e}) nonfinite {int((~torch.isfinite(g[k])).sum())}')
        print(f'run {run}: {"bit-identical" if not bad else f"{len(bad)} differences"}', flush=True)
        for line in bad[:40]:
            print('   ', line, flush=True)


if __name__ == '__main__':
    main()
