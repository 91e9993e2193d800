"""Diagnostic (not collected by pytest): one DoubleConv forward/backward, HIP stages vs torch CPU autograd.

    python tests/diag_dc.py
"""
import os
import sys

import numpy as np
import torch

import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from multimodal_siamese_cd_amd import engine, hip  # noqa: E402
from multimodal_siamese_cd_amd.utils.networks import DoubleConv  # noqa: E402


def rel(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def nhwc(t):
    return t.detach().permute(0, 2, 3, 1).contiguous()


def run(n, h, w, cin_real, cpad, cout, nseg, seed=0):
    torch.manual_seed(seed)
    dev = torch.device('cuda:0')
    dc = DoubleConv(cin_real, cout)
    with torch.no_grad():
        for p in dc.parameters():
            p.uniform_(-0.3, 0.3)
        dc.conv[1].weight.add_(1.0)
        dc.conv[4].weight.add_(1.0)
    x = torch.rand(n, cin_real, h, w)
    g = torch.randn(n, cout, h, w)
    # CPU reference with retained intermediates (per-segment BN batches)
    P = {k: v.detach().clone().requires_grad_(True) for k, v in dc.named_parameters()}
    per = n // nseg

    def bn_relu(t, key):
        outs = []
        for s in range(nseg):
            rm, rv = torch.zeros(t.shape[1]), torch.ones(t.shape[1])
            outs.append(F.relu(F.batch_norm(t[s * per:(s + 1) * per], rm, rv, P[key + '.weight'], P[key + '.bias'],
                                            True, 0.1, 1e-5)))
        return torch.cat(outs)

    y0 = F.conv2d(x, P['conv.0.weight'], P['conv.0.bias'], padding=1)
    y0.retain_grad()
    a0 = bn_relu(y0, 'conv.1')
    a0.retain_grad()
    y1 = F.conv2d(a0, P['conv.3.weight'], P['conv.3.bias'], padding=1)
    y1.retain_grad()
    a1 = bn_relu(y1, 'conv.4')
    a1.backward(g)

    dcd = dc.to(dev)
    xp = torch.empty(n, h, w, cpad, device=dev)
    xd = x.to(dev)
    hip.pack_nchw(xd, 0, cin_real, xp)
    a1h, saved, *_ = engine._dc_forward(xp, dcd, nseg, True, True)
    gd = nhwc(g).to(dev)
    xs, y0h, a0h, st0, y1h, st1 = saved[:6]
    print(f'n={n} {h}x{w} cin={cin_real}(pad {cpad}) cout={cout} nseg={nseg}')
    print(f'  fwd  y0 {rel(y0h.cpu(), nhwc(y0)):.1e} a0 {rel(a0h.cpu(), nhwc(a0)):.1e} y1 {rel(y1h.cpu(), nhwc(y1)):.1e}'
          f' a1 {rel(a1h.cpu(), nhwc(a1)):.1e}')
    conv0, bn0, conv1, bn1 = dcd.conv[0], dcd.conv[1], dcd.conv[3], dcd.conv[4]
    dy1, dg1, db1, dbias1 = engine._bn_backward(y1h, gd, st1, bn1, True)
    print(f'  bn1  dy1 {rel(dy1.cpu(), nhwc(y1.grad)):.1e} dgamma {rel(dg1.cpu(), P["conv.4.weight"].grad):.1e}'
          f' dbeta {rel(db1.cpu(), P["conv.4.bias"].grad):.1e}')
    ga0 = torch.empty(dy1.shape[:3] + (conv1.in_channels,), device=dev)
    hip.conv_igemm(hip.nhwc(dy1), dy1.shape[1], dy1.shape[2], 1, hip.TAPS_3X3, hip.pack_conv3x3(conv1.weight.detach(), 1),
                   conv1.in_channels, None, hip.nhwc(ga0))
    print(f'  dX1  ga0 {rel(ga0.cpu(), nhwc(a0.grad)):.1e}')
    gw1 = engine._wgrad3x3(dy1, a0h, conv1.weight)
    print(f'  dW1  {rel(gw1.cpu(), P["conv.3.weight"].grad):.1e}')
    dy0, dg0, db0, dbias0 = engine._bn_backward(y0h, ga0, st0, bn0, True)
    print(f'  bn0  dy0 {rel(dy0.cpu(), nhwc(y0.grad)):.1e} dgamma {rel(dg0.cpu(), P["conv.1.weight"].grad):.1e}'
          f' dbeta {rel(db0.cpu(), P["conv.1.bias"].grad):.1e}')
    # feed the exact reference ga0 to isolate BN0 backward
    ga0_ref = nhwc(a0.grad).to(dev)
    dy0b, dg0b, db0b, _ = engine._bn_backward(y0h, ga0_ref, st0, bn0, True)
    print(f'  bn0 (ref ga0) dy0 {rel(dy0b.cpu(), nhwc(y0.grad)):.1e} dgamma {rel(dg0b.cpu(), P["conv.1.weight"].grad):.1e}'
          f' dbeta {rel(db0b.cpu(), P["conv.1.bias"].grad):.1e}')
    gw0 = engine._wgrad3x3(dy0, xp, conv0.weight)
    print(f'  dW0  {rel(gw0.cpu(), P["conv.0.weight"].grad):.1e}')
    gw0b = engine._wgrad3x3(nhwc(y0.grad).to(dev), xp, conv0.weight)
    print(f'  dW0 (ref dy0) {rel(gw0b.cpu(), P["conv.0.weight"].grad):.1e}')
    mask_h = (y0h * st0.scale.view(1, 1, 1, -1)[..., :] if nseg == 1 else None)
    # mask agreement between HIP forward and CPU forward
    am = (a0h.cpu() > 0)
    bm = (nhwc(a0) > 0)
    print(f'  relu-mask mismatches a0: {(am != bm).sum().item()} of {am.numel()}')
    am1 = (a1h.cpu() > 0)
    bm1 = (nhwc(a1) > 0)
    print(f'  relu-mask mismatches a1: {(am1 != bm1).sum().item()} of {am1.numel()}')


if __name__ == "__main__" and len(sys.argv) == 1:
    hip.load_library()
    run(4, 64, 64, 5, 8, 8, 2)
    run(4, 64, 64, 8, 8, 8, 2)
    run(2, 64, 64, 8, 8, 8, 1)
    run(4, 16, 16, 8, 8, 8, 2)
    run(4, 64, 64, 16, 16, 16, 2)


def run_fixture(name='siamese_t8-16'):
    """The inc block of a fixture with its exact inputs/weights; incoming grad = oracle's level-0 feature grad."""
    from oracle import siamese_oracle as O
    from oracle.golden import Fixture
    dev = torch.device('cuda:0')
    fx = Fixture(name)
    topo = fx.cfg['TOPOLOGY']
    P = {k: torch.from_numpy(v.copy()).requires_grad_(True) for k, v in fx.params0.items()}
    B = O.fresh_buffers(O.param_shapes(fx.model_type, fx.cfg))
    batch = fx.batch()
    f1 = O.encoder(batch['x_t1'], P, B, 'inc.', 'encoder.', topo, True)[::-1]
    f2 = O.encoder(batch['x_t2'], P, B, 'inc.', 'encoder.', topo, True)[::-1]
    for t in f1 + f2:
        t.retain_grad()
    od = O.diff(f1, f2)
    odec = O.decoder(od[::-1], P, B, 'decoder.', topo, True)
    O.power_jaccard_loss(O.out_conv(odec, P, 'outc.'), batch['y_change']).backward()
    g0 = torch.cat([f1[0].grad, f2[0].grad])
    # CPU inc block with retained intermediates
    x = torch.cat([batch['x_t1'], batch['x_t2']])
    Q = {k[len('inc.conv.'):]: v.detach().clone().requires_grad_(True) for k, v in P.items() if k.startswith('inc.')}
    n = x.shape[0]
    per = n // 2

    def bn_relu(t, key, keep):
        outs = []
        for s in range(2):
            z = F.batch_norm(t[s * per:(s + 1) * per], torch.zeros(t.shape[1]), torch.ones(t.shape[1]),
                             Q[key + '.weight'], Q[key + '.bias'], True, 0.1, 1e-5)
            keep.append(z)
            outs.append(F.relu(z))
        return torch.cat(outs)

    z0, z1 = [], []
    y0 = F.conv2d(x, Q['conv.0.weight'], Q['conv.0.bias'], padding=1)
    y0.retain_grad()
    a0 = bn_relu(y0, 'conv.1', z0)
    a0.retain_grad()
    y1 = F.conv2d(a0, Q['conv.3.weight'], Q['conv.3.bias'], padding=1)
    a1 = bn_relu(y1, 'conv.4', z1)
    a1.backward(g0)
    print('fixture', name, 'ref-vs-golden dgamma0', rel(Q['conv.1.weight'].grad, fx.grads['inc.conv.conv.1.weight']),
          'dW0', rel(Q['conv.0.weight'].grad, fx.grads['inc.conv.conv.0.weight']))
    zz0 = torch.cat(z0).detach()
    print('  |z0| min', zz0.abs().min().item(), ' count |z0|<1e-6:', (zz0.abs() < 1e-6).sum().item(),
          ' exact zeros:', (zz0 == 0).sum().item())
    zz1 = torch.cat(z1).detach()
    print('  |z1| min', zz1.abs().min().item(), ' count |z1|<1e-6:', (zz1.abs() < 1e-6).sum().item())

    from multimodal_siamese_cd_amd.utils.networks import DoubleConv
    dc = DoubleConv(5, topo[0])
    with torch.no_grad():
        for k, p in dc.named_parameters():
            p.copy_(Q[k])
    dcd = dc.to(dev)
    xp = torch.empty(n, x.shape[2], x.shape[3], 8, device=dev)
    xd = x.to(dev)
    hip.pack_nchw(xd, 0, 5, xp)
    a1h, saved, *_ = engine._dc_forward(xp, dcd, 2, True, True)
    xs, y0h, a0h, st0, y1h, st1 = saved[:6]
    am, bm = (a0h.cpu() > 0), (nhwc(a0) > 0)
    bad = (am != bm).nonzero()
    print('  a0 mask mismatches', bad.shape[0], 'z at mismatches', nhwc(torch.cat(z0))[am != bm][:8].tolist())
    print('  a0 hip at mismatches', a0h.cpu()[am != bm][:8].tolist())
    gd = nhwc(g0).to(dev)
    gx, pg = engine._dc_backward(gd, saved, dcd, need_dx=False)
    names = ['conv.0.weight', 'conv.0.bias', 'conv.1.weight', 'conv.1.bias', 'conv.3.weight', 'conv.3.bias',
             'conv.4.weight', 'conv.4.bias']
    for nm, gg in zip(names, pg):
        print(f'  {nm:16s} hip-vs-cpu {rel(gg.cpu(), Q[nm].grad):.1e}')


if __name__ == '__main__' and len(sys.argv) > 1:
    run_fixture(sys.argv[1])
