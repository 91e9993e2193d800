"""Per-layer timing of the BatchNorm / elementwise kernels of the bench workload (SiameseUNet 256^2, bs=32).

    python tools/perf_bn.py [--batch 32] [--reps 5] [--storage bf16]

For every conv output of one training step, times scd_bn_train_stats, scd_bn_relu_apply and
scd_bn_relu_backward with HIP events.  Prints the achieved HBM rate from the algorithmic bytes:
4, 8 and 20 B/elem respectively (the backward reads y and da twice and writes dy); half of that with
--storage bf16 (bf16 activations and gradients, the bf16 configs' ACT_STORAGE).
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from multimodal_siamese_cd_amd import hip  # noqa: E402
from perf_conv import layers, timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=32)
    ap.add_argument('--reps', type=int, default=5)
    ap.add_argument('--storage', choices=('f32', 'bf16'), default='f32')
    args = ap.parse_args()
    dt = torch.bfloat16 if args.storage == 'bf16' else torch.float32
    eb = 2 if args.storage == 'bf16' else 4
    hip.load_library()
    dev = torch.device('cuda:0')
    # streaming references on the largest map: torch's float4 copy (1 read + 1 write) and add (2 reads + 1 write)
    big = torch.randn(args.batch * 65536 * 64, device=dev)
    big2, out = torch.randn_like(big), torch.empty_like(big)
    t_c = timeit(lambda: out.copy_(big), args.reps)
    t_add = timeit(lambda: torch.add(big, big2, out=out), args.reps)
    print(f'torch copy {t_c:.3f} ms {8 * big.numel() / t_c / 1e9:.2f} TB/s | add {t_add:.3f} ms '
          f'{12 * big.numel() / t_add / 1e9:.2f} TB/s  ({big.numel() / 1e6:.0f} M floats)', flush=True)
    del big, big2, out
    # the input packing (NCHW 5 bands -> NHWC 16 channels), without and with the h2 input bound
    xin = torch.rand(args.batch, 5, 256, 256, device=dev)
    xpk = torch.empty(args.batch, 256, 256, 16, device=dev)
    bnd = torch.zeros(1, device=dev)
    t_p = timeit(lambda: hip.pack_nchw(xin, 0, 5, xpk), args.reps)
    t_pb = timeit(lambda: hip.pack_nchw(xin, 0, 5, xpk, bound=bnd), args.reps)
    pb = 4 * (xin.numel() + xpk.numel())
    print(f'pack_nchw {t_p:.3f} ms {pb / t_p / 1e9:.2f} TB/s | with bound {t_pb:.3f} ms {pb / t_pb / 1e9:.2f} TB/s '
          f'(bound {bnd.item():.6f} vs max {xin.max().item():.6f})', flush=True)
    del xin, xpk
    tot = {'stats': 0.0, 'apply': 0.0, 'bwd': 0.0}
    byt = {'stats': 0.0, 'apply': 0.0, 'bwd': 0.0}
    print(f'{"layer":8s} {"n":>3s} {"hw":>4s} {"c":>5s} | {"stats ms":>8s} {"TB/s":>5s} | {"apply ms":>8s} {"TB/s":>5s} | '
          f'{"bwd ms":>8s} {"TB/s":>5s}')
    for name, n, s, _, co in layers(args.batch):
        nseg = 2 if name.startswith('enc') else 1
        y = torch.randn(n, s, s, co, device=dev, dtype=dt)
        da = torch.randn(n, s, s, co, device=dev, dtype=dt)
        a = torch.empty_like(y)
        dy = torch.empty_like(y)
        gamma = torch.rand(co, device=dev) + 0.5
        beta = torch.randn(co, device=dev)
        rm, rv = torch.zeros(co, device=dev), torch.ones(co, device=dev)
        sm, si = torch.empty(nseg * co, device=dev), torch.empty(nseg * co, device=dev)
        sc, sh = torch.empty(nseg * co, device=dev), torch.empty(nseg * co, device=dev)
        dg, db, dbias = torch.empty(co, device=dev), torch.empty(co, device=dev), torch.empty(co, device=dev)
        ws = torch.empty(hip.bn_workspace_bytes(n, s, s, co, nseg), dtype=torch.uint8, device=dev)
        Y, A, DA, DY = hip.nhwc(y), hip.nhwc(a), hip.nhwc(da), hip.nhwc(dy)
        el = y.numel()
        t_s = timeit(lambda: hip.bn_train_stats(Y, nseg, gamma, beta, 1e-5, 0.1, False, rm, rv, sm, si, sc, sh, ws),
                     args.reps)
        t_a = timeit(lambda: hip.bn_relu_apply(Y, nseg, sc, sh, A), args.reps)
        t_b = timeit(lambda: hip.bn_relu_backward(Y, DA, nseg, sm, si, gamma, sc, sh, dg, db, dbias, DY, ws),
                     args.reps)
        cells = []
        for k, t, b in (('stats', t_s, eb), ('apply', t_a, 2 * eb), ('bwd', t_b, 5 * eb)):
            tot[k] += t
            byt[k] += b * el
            cells.append(f'{t:8.3f} {b * el / t / 1e9:5.2f}')
        print(f'{name:8s} {n:3d} {s:4d} {co:5d} | ' + ' | '.join(cells), flush=True)
    for k in tot:
        print(f'{k:6s} total {tot[k]:8.2f} ms  {byt[k] / tot[k] / 1e9:5.2f} TB/s')
    # the encoder levels' backward: da = maxpool_bwd(gy, idx) -/+ the Siamese difference gradient, formed on the fly
    # (scd_bn_relu_backward_pooled, the pair kernels); algorithmic bytes per y element: 2 x (y 4 + difference 2 (one
    # t1/t2 pair reads it once) + pooled gradient 1 + argmax 0.25) + dy 4 = 18.5 (fp32; bf16 storage: 9.5)
    print(f'{"level":8s} {"n":>3s} {"hw":>4s} {"c":>5s} | {"pooled bwd ms":>13s} {"TB/s":>5s}')
    tp, bp = 0.0, 0.0
    for name, n, s, _, co in layers(args.batch):
        if not (name.startswith('enc') and name.endswith('b')):
            continue
        y = torch.randn(n, s, s, co, device=dev, dtype=dt)
        gy = torch.randn(n, s // 2, s // 2, co, device=dev, dtype=dt)
        idx = torch.randint(0, 4, (n, s // 2, s // 2, co), device=dev, dtype=torch.uint8)
        cat = torch.randn(n // 2, s, s, 2 * co, device=dev, dtype=dt)
        dy = torch.empty_like(y)
        gamma = torch.rand(co, device=dev) + 0.5
        sm, si = torch.randn(2 * co, device=dev), torch.rand(2 * co, device=dev) + 0.5
        sc, sh = torch.rand(2 * co, device=dev), torch.randn(2 * co, device=dev)
        dg, db, dbias = torch.empty(co, device=dev), torch.empty(co, device=dev), torch.empty(co, device=dev)
        ws = torch.empty(hip.bn_workspace_bytes(n, s, s, co, 2), dtype=torch.uint8, device=dev)
        t = timeit(lambda: hip.bn_relu_backward_pooled(hip.nhwc(y), hip.nhwc(gy), idx, hip.nhwc(cat, 0, co), 1, 2, sm,
                                                       si, gamma, sc, sh, dg, db, dbias, hip.nhwc(dy), ws), args.reps)
        b = (18.5 if eb == 4 else 9.5) * y.numel()
        tp += t
        bp += b
        print(f'{name:8s} {n:3d} {s:4d} {co:5d} | {t:13.3f} {b / t / 1e9:5.2f}', flush=True)
    print(f'pooled total {tp:8.2f} ms  {bp / tp / 1e9:5.2f} TB/s')


if __name__ == '__main__':
    main()
