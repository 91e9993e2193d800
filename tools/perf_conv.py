"""Per-shape timing of the MFMA conv kernels for the bench workload (SiameseUNet 256^2, bs=32, fp32).

    python tools/perf_conv.py [--batch 32] [--reps 5] [--only fwd|dgrad|wgrad]

Times every 3x3 conv of one training step (forward, data-grad, weight-grad) and the ConvTranspose GEMMs
with HIP events, prints TF/s against the 157.3 TF/s fp32 MFMA peak and the step total.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from multimodal_siamese_cd_amd import hip  # noqa: E402

PEAK = 157.3


def layers(batch, size=256, topo=(64, 128, 256, 512), cin=8):
    L = len(topo)
    ch = [topo[0]] + [topo[i + 1] if i != L - 1 else topo[i] for i in range(L)]
    out = []
    for lvl in range(L + 1):
        s = size >> lvl
        c_in = cin if lvl == 0 else ch[lvl - 1]
        out.append((f'enc{lvl}a', 2 * batch, s, c_in, ch[lvl]))
        out.append((f'enc{lvl}b', 2 * batch, s, ch[lvl], ch[lvl]))
    for idx in reversed(range(L)):
        s = size >> idx
        c = ch[idx]
        o = ch[idx - 1] if idx != 0 else ch[0]
        out.append((f'up{idx + 1}a', batch, s, 2 * c, o))
        out.append((f'up{idx + 1}b', batch, s, o, o))
    return out


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=32)
    ap.add_argument('--reps', type=int, default=5)
    ap.add_argument('--only', default=None)
    ap.add_argument('--layer', default=None, help='run only this layer name (e.g. enc1b)')
    ap.add_argument('--cin', type=int, default=None,
                    help='input-layer channels as stored (default: the model\'s padding of 5 bands, engine.pad_in)')
    ap.add_argument('--math', default=None, choices=['f32', 'x3', 'x5', 'bf16', 'h2'],
                    help='conv arithmetic (default: library default; h2 gets absmax operand bounds)')
    ap.add_argument('--storage', default='fp32', choices=['fp32', 'bf16'],
                    help='activation / gradient storage of the operands (bf16: the bf16 configs, with --math bf16)')
    ap.add_argument('--variants', default=None,
                    help='comma-separated variants, interleaved per layer; a variant is "+"-joined settings '
                         'h16=<hip.set_halo16 mode> or tune=<SCD_TUNE_* bits, OR-ed>, e.g. h16=1+tune=0x100000,h16=1')
    args = ap.parse_args()
    hip.load_library()
    if args.math:
        hip.set_conv_math(args.math)
    print(f'conv math: {hip.conv_math()}')
    dev = torch.device('cuda:0')
    modes = [None] if args.variants is None else args.variants.split(',')
    tots = {m: {'fwd': [0.0, 0.0], 'dgrad': [0.0, 0.0], 'wgrad': [0.0, 0.0]} for m in modes}
    print(f'{"layer":8s} {"n":>3s} {"hw":>4s} {"cin":>5s} {"cout":>5s} | '
          f'{"fwd ms":>8s} {"TF/s":>6s} | {"dgrad ms":>8s} {"TF/s":>6s} | {"wgrad ms":>8s} {"TF/s":>6s}')
    from multimodal_siamese_cd_amd import engine
    cin = args.cin or engine.pad_in(5)
    for name, n, s, ci, co in layers(args.batch, cin=cin):
        if args.layer and name != args.layer:
            continue
        sdt = torch.bfloat16 if args.storage == 'bf16' else torch.float32
        x = torch.randn(n, s, s, ci, device=dev).to(sdt)
        dy = torch.randn(n, s, s, co, device=dev).to(sdt)
        w = torch.randn(co, ci, 3, 3, device=dev) * 0.05
        y = torch.empty(n, s, s, co, device=dev, dtype=sdt)
        dx = torch.empty(n, s, s, ci, device=dev, dtype=sdt)
        wf = hip.pack_conv3x3(w, 0)
        wb = hip.pack_conv3x3(w, 1)
        flops = 2.0 * n * s * s * co * 9 * ci
        xb = db = None
        if hip.conv_math() == 'h2':  # the operand bounds the engine's producers would supply
            xb, db = torch.zeros(1, device=dev), torch.zeros(1, device=dev)
            hip.absmax_bound(hip.nhwc(x), xb)
            hip.absmax_bound(hip.nhwc(dy), db)
        for mode in modes:
            if mode is not None:  # every variant starts from tune 0
                hip.set_tune(0)
                for kv in mode.split('+'):
                    k, v = kv.split('=')
                    if k == 'h16':
                        hip.set_halo16(int(v))
                    elif k == 'tune':
                        hip.set_tune(hip.get_tune() | int(v, 0))
                    else:
                        raise SystemExit(f'unknown setting {k}')
            tot = tots[mode]
            res = {}
            if args.only in (None, 'fwd'):
                res['fwd'] = timeit(lambda: hip.conv_igemm(hip.nhwc(x), s, s, 1, hip.TAPS_3X3, wf, co, None,
                                                           hip.nhwc(y), src_bound=xb), args.reps)
            if args.only in (None, 'dgrad') and not name.startswith('enc0a'):
                res['dgrad'] = timeit(lambda: hip.conv_igemm(hip.nhwc(dy), s, s, 1, hip.TAPS_3X3, wb, ci, None,
                                                             hip.nhwc(dx), src_bound=db), args.reps)
            if args.only in (None, 'wgrad'):
                d, nsplit, nbytes = hip.wgrad_plan(hip.nhwc(dy), hip.nhwc(x), 1, hip.TAPS_3X3, None, db, xb)
                slabs = torch.empty(nbytes // 4, device=dev)
                res['wgrad'] = timeit(lambda: hip.conv_wgrad(d, slabs), args.reps)
            cells = []
            for k in ('fwd', 'dgrad', 'wgrad'):
                if k in res:
                    t = res[k]
                    tot[k][0] += t
                    tot[k][1] += flops
                    cells.append(f'{t:8.3f} {flops / t / 1e9:6.1f}')
                else:
                    cells.append(f'{"-":>8s} {"-":>6s}')
            tag = name if mode is None else f'{name}/{mode}'
            print(f'{tag:8s} {n:3d} {s:4d} {ci:5d} {co:5d} | ' + ' | '.join(cells), flush=True)
    for mode, tot in tots.items():
        if mode is not None:
            print(f'-- variant {mode}')
        allt = sum(v[0] for v in tot.values())
        allf = sum(v[1] for v in tot.values())
        for k, (t, f) in tot.items():
            if t:
                print(f'{k:6s} total {t:8.2f} ms  {f / t / 1e9:6.1f} TF/s  ({f / t / 1e9 / PEAK * 100:.1f}% of fp32 peak)')
        print(f'3x3 total {allt:8.2f} ms  {allf / allt / 1e9:6.1f} TF/s  ({allf / allt / 1e9 / PEAK * 100:.1f}% of peak)')

if __name__ == '__main__':
    main()
