"""Repeat one halo weight-grad case (tests/test_kernels_gpu.py::test_wgrad_halo_variants) and report mismatches
against the fp32 reference, with the rows / taps / channels of the wrong elements (flake hunt).

    python tools/flake_wgrad.py [--reps 200] [--variant 0] [--shape 3,6,16,128,192]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from multimodal_siamese_cd_amd import hip  # noqa: E402


def nchw(t):
    return t.permute(0, 3, 1, 2).contiguous()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--reps', type=int, default=200)
    ap.add_argument('--variant', type=int, default=0)
    ap.add_argument('--shape', default='3,6,16,128,192')
    ap.add_argument('--fill', type=float, default=float('nan'), help='slab workspace fill before each run')
    args = ap.parse_args()
    n, h, w, ci, co = map(int, args.shape.split(','))
    hip.load_library()
    dev = torch.device('cuda:0')
    hip.set_conv_math('x3')
    hip.set_wgrad16(args.variant)
    g = torch.Generator().manual_seed(5 * args.variant + ci + co + h)
    x = torch.randn(n, h, w, ci, generator=g)
    dy = torch.randn(n, h, w, co, generator=g)
    ref = torch.nn.grad.conv2d_weight(nchw(x), (co, ci, 3, 3), nchw(dy), padding=1).to(dev)
    xd, dyd = x.to(dev), dy.to(dev)
    bad = 0
    for r in range(args.reps):
        d, nsplit, nbytes = hip.wgrad_plan(hip.nhwc(dyd), hip.nhwc(xd), 1, hip.TAPS_3X3)
        slabs = torch.full((nbytes // 4,), args.fill, device=dev)
        hip.conv_wgrad(d, slabs)
        dw = torch.empty(co, ci, 3, 3, device=dev)
        hip.wgrad_finalize(slabs, nsplit, co, 9, ci, 0, ci, dw)
        err = ((dw - ref).abs() > 1e-3 * ref.abs().max()) | ~torch.isfinite(dw)
        if err.any():
            bad += 1
            idx = err.nonzero()
            print(f'rep {r}: {int(err.sum())} wrong, nsplit {nsplit}, rows {sorted(set(idx[:, 0].tolist()))[:12]} '
                  f'ch {sorted(set(idx[:, 1].tolist()))[:12]} taps {sorted(set((idx[:, 2] * 3 + idx[:, 3]).tolist()))}',
                  flush=True)
            sl = slabs.view(nsplit, co, 9, ci)
            print('  non-finite slab entries per split:', (~torch.isfinite(sl)).flatten(1).sum(1).tolist()[:32],
                  flush=True)
    print(f'{bad} of {args.reps} runs wrong', flush=True)


if __name__ == '__main__':
    main()
