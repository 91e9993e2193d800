"""Bitwise equivalence of two h2 tile layouts of the halo conv on every epilogue / operand option.

    python tools/tile_equiv.py [--env SCD_H2_TILE64=0]

Each case runs twice in one process, with the library's default choice and with `--env` set (read by libscd at
launch).  The per-output accumulation order is the same in both layouts, so outputs, BatchNorm statistic records,
BatchNorm-backward records and raised bounds must be bit-identical.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from multimodal_siamese_cd_amd import hip  # noqa: E402
from multimodal_siamese_cd_amd.hip import TAPS_3X3, nhwc  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--env', default='SCD_H2_TILE64=0')
    args = ap.parse_args()
    key, val = args.env.split('=')
    hip.load_library()
    dev = torch.device('cuda:0')
    hip.set_conv_math('h2')
    g = torch.Generator(device=dev).manual_seed(11)
    bad = 0
    for n, h, w, ci, co, ldc_s, ldc_d, mode in [
            (2, 32, 32, 64, 64, 64, 64, 'plain'), (2, 32, 32, 32, 64, 32, 64, 'plain'),
            (4, 32, 32, 64, 64, 64, 64, 'stats'), (4, 32, 32, 64, 64, 64, 64, 'in_bn'),
            (2, 32, 32, 64, 64, 64, 64, 'bn_bwd'), (2, 32, 32, 32, 64, 32, 64, 'bn_bwd'),
            (2, 32, 32, 64, 64, 96, 64, 'plain'), (2, 32, 32, 32, 64, 32, 128, 'dst_bound'),
            (2, 64, 64, 128, 64, 128, 64, 'bn_bwd'), (2, 16, 48, 64, 96, 64, 96, 'plain')]:
        base = torch.randn(n, h, w, ldc_s, device=dev, generator=g)
        src_t = base[..., ldc_s - ci:]
        wt = torch.randn(co, ci, 3, 3, device=dev, generator=g) / (3 * ci ** 0.5)
        wpk = hip.pack_conv3x3(wt, 0)
        bound = src_t.abs().max().reshape(1).clone() * (2.0 if mode == 'in_bn' else 1.0)
        nseg = 2
        sc = torch.rand(nseg * ci, device=dev, generator=g) + 0.5
        sh = torch.randn(nseg * ci, device=dev, generator=g) * 0.1
        yb = torch.randn(n, h, w, co, device=dev, generator=g)
        mu, iv = torch.randn(nseg * co, device=dev, generator=g) * 0.1, torch.rand(nseg * co, device=dev) + 0.5
        bsc, bsh = torch.rand(nseg * co, device=dev) + 0.5, torch.randn(nseg * co, device=dev) * 0.1
        outs = []
        for setting in (None, val):
            if setting is None:
                os.environ.pop(key, None)
            else:
                os.environ[key] = setting
            dstb = torch.empty(n, h, w, ldc_d, device=dev).fill_(7.0)
            dst = dstb[..., ldc_d - co:]
            src = nhwc(src_t)
            extra, rec, dbound = {}, None, None
            if mode == 'in_bn':
                extra['in_bn'] = (sc, sh, nseg)
                assert hip.igemm_input_bn_supported(src, h, w, 1, TAPS_3X3, wpk, co, nhwc(dst), extra['in_bn'], bound)
            if mode == 'stats':
                nt, _ = hip.igemm_stat_tiles(src, h, w, 1, TAPS_3X3, wpk, co, nhwc(dst), src_bound=bound)
                assert nt
                rec = torch.full((nt * co * 2,), 9.0, device=dev)
                extra['stat_rec'] = rec
            if mode == 'bn_bwd':
                nt, _ = hip.igemm_bn_bwd_tiles(src, h, w, 1, TAPS_3X3, wpk, co, nhwc(dst), bound)
                assert nt
                rec = torch.full((co * nt * 2,), 9.0, device=dev)
                extra['bn_bwd'] = (yb, nseg, mu, iv, bsc, bsh, rec)
            if mode == 'dst_bound':
                dbound = torch.zeros(1, device=dev)
                extra['dst_bound'] = dbound
            hip.conv_igemm(src, h, w, 1, TAPS_3X3, wpk, co, None, nhwc(dst), src_bound=bound, **extra)
            torch.cuda.synchronize()
            outs.append([dstb.clone()] + ([rec.clone()] if rec is not None else []) +
                        ([dbound.clone()] if dbound is not None else []))
        os.environ.pop(key, None)
        same = all(torch.equal(a, b) for a, b in zip(*outs))
        if not same:
            bad += 1
            diffs = [(int((a != b).sum()), a.numel(), f'{float((a - b).abs().max() / b.abs().max().clamp_min(1e-30)):.1e}')
                     for a, b in zip(*outs)]
            print(f'DIFFER n{n} {h}x{w} ci{ci} co{co} ldc {ldc_s}/{ldc_d} {mode}: (differing, total, max|d|/max|ref|) per output {diffs}',
                  flush=True)
        else:
            print(f'same   n{n} {h}x{w} ci{ci} co{co} ldc {ldc_s}/{ldc_d} {mode}', flush=True)
    print(f'{bad} cases differ', flush=True)


if __name__ == '__main__':
    main()
