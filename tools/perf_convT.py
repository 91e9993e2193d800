"""Per-level timing of the decoder's ConvTranspose2d(2, s2) GEMMs (forward: 1 tap into the pixel-shuffled concat
slice; data grad: 4 taps, stride 2): the per-tap x3 kernel under tile variants (SCD_TUNE_X3_TILE), or with --math h2 the
gather16 kernel (source bounds given; --dst-bound also raises the concat bound in the forward, as the engine does).

    python tools/perf_convT.py [--batch 32] [--reps 10] [--tiles 0,1,2,4,5] [--math h2] [--dst-bound] [--plain]

Tile 0 is the library's own choice.  HIP events, interleaved per level.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from multimodal_siamese_cd_amd import hip  # noqa: E402


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=32)
    ap.add_argument('--reps', type=int, default=10)
    ap.add_argument('--tiles', default='0,1,2,4,5')
    ap.add_argument('--plain', action='store_true', help='also time the forward GEMM with plain stores')
    ap.add_argument('--math', default='x3', choices=['x3', 'h2'])
    ap.add_argument('--dst-bound', action='store_true', help='forward raises a dst bound (h2 engine path)')
    ap.add_argument('--tunes', default=None, help='comma list of raw SCD_TUNE_* values to compare instead of --tiles '
                                                  '(e.g. 0,0x40000000)')
    args = ap.parse_args()
    hip.load_library()
    hip.set_conv_math(args.math)
    dev = torch.device('cuda:0')
    tiles = args.tunes.split(',') if args.tunes else args.tiles.split(',')
    tune_of = (lambda t: int(t, 0)) if args.tunes else (lambda t: hip.tune_x3_tile(int(t)))
    # (level, input size, ConvT channels (in == out, networks.py Up), skip channels) of SiameseUNet [64,128,256,512]
    # at 256^2
    levels = [('up4', 16, 512, 512, 512), ('up3', 32, 256, 256, 256), ('up2', 64, 128, 128, 128),
              ('up1', 128, 64, 64, 64)]
    tot = {t: [0.0, 0.0] for t in tiles}
    for name, hc, ci, co, cs in levels:
        b = args.batch
        x = torch.randn(b, hc, hc, ci, device=dev)
        wt = torch.randn(ci, co, 2, 2, device=dev) * 0.05
        bias = torch.randn(co, device=dev)
        cat = torch.empty(b, 2 * hc, 2 * hc, cs + co, device=dev)
        gx = torch.empty(b, hc, hc, ci, device=dev)
        wf, wb = hip.pack_convT2x2(wt, 0), hip.pack_convT2x2(wt, 1)
        gup = hip.nhwc(cat, cs, co)
        xb = gb = db = None
        if args.math == 'h2':
            cat.normal_()
            xb, gb = torch.zeros(1, device=dev), torch.zeros(1, device=dev)
            hip.absmax_bound(hip.nhwc(x), xb)
            hip.absmax_bound(hip.nhwc(cat), gb)
            if args.dst_bound:
                db = torch.zeros(1, device=dev)
        for t in tiles:
            hip.set_tune(tune_of(t))  # tiles: 0 = automatic
            f = timeit(lambda: hip.conv_igemm(hip.nhwc(x), hc, hc, 1, hip.TAPS_1, wf, 4 * co, bias, gup,
                                              store_mode=1, src_bound=xb, dst_bound=db), args.reps)
            d = timeit(lambda: hip.conv_igemm(gup, hc, hc, 2, hip.TAPS_2X2, wb, ci, None, hip.nhwc(gx), src_bound=gb),
                       args.reps)
            if args.plain:  # same GEMM, plain row-major stores (no pixel shuffle): isolates the epilogue
                flat = torch.empty(b, hc, hc, 4 * co, device=dev)
                fp = timeit(lambda: hip.conv_igemm(hip.nhwc(x), hc, hc, 1, hip.TAPS_1, wf, 4 * co, bias,
                                                   hip.nhwc(flat), src_bound=xb), args.reps)
                print(f'{name} tile {t}: fwd plain-store {fp * 1e3:7.1f} us', flush=True)
            tot[t][0] += f
            tot[t][1] += d
            gb_ = 4 * b * hc * hc * ci * 5 / 1e9  # fp32 bytes: fwd reads x, writes 4x its pixels; dgrad the reverse
            print(f'{name} hc={hc:4d} ci={ci:4d} co={co:4d} {"tune" if args.tunes else "tile"} {t}: fwd {f * 1e3:7.1f} us '
                  f'({gb_ / f:5.2f} TB/s)  dgrad {d * 1e3:7.1f} us ({gb_ / d:5.2f} TB/s)', flush=True)
    hip.set_tune(0)
    for t, (f, d) in tot.items():
        print(f'tile {t}: fwd {f * 1e3:7.1f} us  dgrad {d * 1e3:7.1f} us  sum {(f + d) * 1e3:7.1f} us')


if __name__ == '__main__':
    main()
