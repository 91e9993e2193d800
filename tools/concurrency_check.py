"""Does a weight-grad launch give the same bits when another kernel runs beside it on a second stream?

    python tools/concurrency_check.py [--reps 10] [--math x3|h2] [--shape 64,64,64,128,128]

Reference: wgrad + slab finalize alone.  Then the same launch on stream B while stream A runs (a) torch matmuls on
unrelated buffers, (b) a libscd 3x3 conv (igemm) on unrelated buffers, (c) the same wgrad on unrelated buffers.  A
mismatch under (a) points at the wgrad kernel itself (timing-dependent); only under (b)/(c) at cross-kernel
interference.
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
    ap.add_argument('--reps', type=int, default=10)
    ap.add_argument('--math', default='x3')
    ap.add_argument('--shape', default='64,64,64,128,128', help='n,h,w,cin,cout')
    args = ap.parse_args()
    hip.load_library()
    dev = torch.device('cuda:0')
    hip.set_conv_math(args.math)
    n, h, w, ci, co = map(int, args.shape.split(','))
    g = torch.Generator(device=dev).manual_seed(3)
    x = torch.randn(n, h, w, ci, device=dev, generator=g)
    dy = torch.randn(n, h, w, co, device=dev, generator=g)
    h2 = args.math == 'h2'
    xb = x.abs().max().reshape(1).clone() if h2 else None
    db = dy.abs().max().reshape(1).clone() if h2 else None

    def wgrad(dy_, x_):
        d, nsplit, nbytes = hip.wgrad_plan(nhwc(dy_), nhwc(x_), 1, TAPS_3X3, None, db, xb)
        slabs = torch.empty(nbytes // 4, device=dev)
        hip.conv_wgrad(d, slabs)
        out = torch.empty(co, ci, 3, 3, device=dev)
        hip.wgrad_finalize(slabs, nsplit, co, 9, ci, 0, ci, out)
        return out

    ref = wgrad(dy, x)
    torch.cuda.synchronize()
    for _ in range(3):
        again = wgrad(dy, x)
        torch.cuda.synchronize()
        print('serial repeat identical:', torch.equal(again, ref), flush=True)

    # unrelated workloads for stream A
    big = torch.randn(8192, 8192, device=dev)
    x2 = torch.randn(n, h, w, ci, device=dev)
    dy2 = torch.randn(n, h, w, co, device=dev)
    wpk = hip.pack_conv3x3(torch.randn(co, ci, 3, 3, device=dev), 0)
    y2 = torch.empty(n, h, w, co, device=dev)

    def side_a(kind):
        if kind == 'matmul':
            for _ in range(4):
                big @ big
        elif kind == 'igemm':
            for _ in range(6):
                hip.conv_igemm(nhwc(x2), h, w, 1, TAPS_3X3, wpk, co, None, nhwc(y2))
        else:
            for _ in range(3):
                wgrad(dy2, x2)

    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    for kind in ('matmul', 'igemm', 'wgrad'):
        bad = 0
        for r in range(args.reps):
            torch.cuda.synchronize()
            with torch.cuda.stream(sa):
                side_a(kind)
            with torch.cuda.stream(sb):
                out = wgrad(dy, x)
            torch.cuda.synchronize()
            if not torch.equal(out, ref):
                bad += 1
                d = (out - ref).abs()
                print(f'  {kind} rep {r}: {int((d > 0).sum())}/{d.numel()} differ, max|d| {float(d.max()):.3e} '
                      f'(max|ref| {float(ref.abs().max()):.3e})', flush=True)
        print(f'{kind:8s} beside the wgrad: {bad} of {args.reps} runs differ', flush=True)


if __name__ == '__main__':
    main()
