"""HIP-event timing of the OutConv 1x1 head forwards (scd_conv1x1_fwd_bn2 / _fwd_bn), on the configs' shapes.

    python tools/perf_head.py [--reps 20]

Cases: the Siamese head (fp32, bs=32, through the last BatchNorm), the dual-task semantic head (fp32, 2 x 64 images,
two BatchNorm segments), DualStream's fusion head (bf16, bs=64, two decoders) and WhateverNet's three heads in one
launch (bf16, bs=16 at 512^2, two decoders).  TB/s counts the bytes read (the activations) plus the logits written.
Round 4 (the bench step, rocprof): Siamese 156 us, DualStream 505 us (2.1 TB/s), WhateverNet 780 us (1.4 TB/s).
Then, per case and source, the head's BatchNorm backward (scd_bn_relu_backward_head with the head's weight grad, the
call HeadsFn makes): TB/s counts y read twice (partial and apply passes), the head gradient read twice, dy written.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from multimodal_siamese_cd_amd import hip  # noqa: E402


def bench(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--reps', type=int, default=20)
    args = ap.parse_args()
    hip.load_library()
    dev = torch.device('cuda:0')
    cases = [('siamese fp32 bs32', torch.float32, 32, 256, 1, 1, 1),
             ('dtsiamese sem fp32 2x64', torch.float32, 128, 256, 1, 1, 2),
             ('dualstream bf16 bs64', torch.bfloat16, 64, 256, 2, 1, 1),
             ('whatevernet bf16 bs16 512^2 x3 heads', torch.bfloat16, 16, 512, 2, 3, 1)]
    for name, dt, n, s, nsrc, nout, nseg in cases:
        ys = [torch.randn(n, s, s, 64, device=dev).to(dt) for _ in range(nsrc)]
        sc = [torch.rand(nseg * 64, device=dev) + 0.5 for _ in range(nsrc)]
        sh = [torch.randn(nseg * 64, device=dev) for _ in range(nsrc)]
        w = torch.randn(nout, 64 * nsrc, device=dev)
        b = torch.randn(nout, device=dev)
        o = torch.empty(n, nout, s, s, device=dev)
        if nsrc == 2:
            fn = lambda: hip.conv1x1_fwd_bn2(hip.nhwc(ys[0]), sc[0], sh[0], hip.nhwc(ys[1]), sc[1], sh[1], nseg, w, b,  # noqa: E731
                                             nout, o)
        else:
            fn = lambda: hip.conv1x1_fwd_bn(hip.nhwc(ys[0]), sc[0], sh[0], nseg, w, b, nout, o)  # noqa: E731
        t = bench(fn, args.reps)
        nbytes = sum(y.numel() * y.element_size() for y in ys) + o.numel() * 4
        print(f'{name:40s} {t * 1e3:8.1f} us  {nbytes / t / 1e9:5.2f} TB/s', flush=True)
        y = ys[0]
        gout = torch.randn(n, nout, s, s, device=dev) * 1e-3
        wh = torch.randn(nout, 64, device=dev)
        sm, si = torch.randn(nseg * 64, device=dev), torch.rand(nseg * 64, device=dev) + 0.5
        gm = torch.rand(64, device=dev) + 0.5
        dg, db, dbias = torch.empty(64, device=dev), torch.empty(64, device=dev), torch.empty(64, device=dev)
        wg = torch.empty(nout, 64, device=dev)
        dy = torch.empty_like(y)
        ws = torch.empty(hip.bn_head_workspace_bytes(n, s, s, 64, nseg, nout), dtype=torch.uint8, device=dev)
        fb = lambda: hip.bn_relu_backward_head(hip.nhwc(y), gout, wh, nout, nseg, sm, si, gm, sc[0], sh[0], dg, db,  # noqa: E731
                                               dbias, hip.nhwc(dy), ws, w_grad=wg)
        tb = bench(fb, args.reps)
        bb = 3 * y.numel() * y.element_size() + 2 * gout.numel() * 4
        print(f'{"  backward (one source, " + str(nout) + " heads)":40s} {tb * 1e3:8.1f} us  {bb / tb / 1e9:5.2f} TB/s',
              flush=True)


if __name__ == '__main__':
    main()
