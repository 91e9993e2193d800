"""HIP-event timing of the OutConv 1x1 head forward on the bench shape ([32, 256, 256, 64] NHWC -> 1 channel).

    python tools/perf_head.py [--reps 20]

Measured (final code): 103-110 us = 4.9-5.2 TB/s with U = 4 pixel sets per wave iteration; U = 8 and 16 were
slower (120, 178 us) in a one-off study.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from multimodal_siamese_cd_amd import hip  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--reps', type=int, default=20)
    ap.add_argument('--batch', type=int, default=32)
    args = ap.parse_args()
    hip.load_library()
    dev = torch.device('cuda:0')
    x = torch.randn(args.batch, 256, 256, 64, device=dev)
    w = torch.randn(1, 64, device=dev)
    b = torch.randn(1, device=dev)
    o = torch.empty(args.batch, 1, 256, 256, device=dev)
    fn = lambda: hip.conv1x1_fwd(hip.nhwc(x), w, b, 1, o)  # noqa: E731
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / args.reps
    print(f'head 1x1 fwd: {t * 1e3:.1f} us, {x.numel() * 4 / t / 1e9:.2f} TB/s')


if __name__ == '__main__':
    main()
