"""A/B of library variants on the bench training step, interleaved in ONE process (guide rule 24).

    python tools/ab_step.py --variants "h16=1,w16=0" "h16=1,w16=1" [--rounds 6 --steps 8]

A variant is a comma list of knob=value with knobs:
  h16   halo16 tile mode (hip.set_halo16: 0 off, 1 auto, 2 + id forced)
  tune  SCD_TUNE_* bits of every conv descriptor (hip.set_tune; decimal or 0x hex)
  fuse  engine BN-apply fusion into the consuming conv (engine.set_options(fuse_input_bn=...))
  fuse_bb  BN-backward partial sums in the data-grad epilogue (engine.set_options(fuse_bn_bwd=...))
  fuse_enc  fused Siamese encoder (engine.set_options(fuse_siamese_encoder=...))
  math  the model's conv arithmetic (model.conv_math: f32 | x3 | x5 | bf16 | h2)
  pack  weight packing: 0 per call, 1 cached per weight, 2 batched per model (engine.packed_conv3x3)
  pool_diff  encoder difference + next-level pooling in one pass (engine.set_options(pool_diff=...))
  pooled_bn_bwd  encoder BN backward forms maxpool_bwd -/+ diff grad on the fly (engine.set_options(...))
  defer_bn_bwd  input layer's BN backward formed inside its weight grad (engine.set_options(defer_bn_bwd=...))
  <engine option>=0|1  any other engine.set_options switch by name (e.g. fuse_head=0)
Prints per-variant median / min ms per step over the rounds.
"""
import argparse
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from multimodal_siamese_cd_amd import engine, hip, trainers  # noqa: E402
from multimodal_siamese_cd_amd.utils import datasets, experiment_manager, networks  # noqa: E402


_DEFAULT_OPTS = dict(engine._OPTS)


def apply(variant: str, model, math0: str):
    """Every variant starts from the defaults: tune bits 0, engine options and the config's arithmetic."""
    hip.set_tune(0)
    model.conv_math = math0
    engine.set_options(**_DEFAULT_OPTS)
    for kv in filter(None, variant.split(',')):
        k, v = kv.split('=')
        if k == 'h16':
            hip.set_halo16(int(v))
        elif k == 'tune':
            hip.set_tune(hip.get_tune() | int(v, 0))
        elif k == 'fuse':
            engine.set_options(fuse_input_bn=bool(int(v)))
        elif k == 'fuse_bb':
            engine.set_options(fuse_bn_bwd=bool(int(v)))
        elif k == 'pack':  # 0 = per-call packing (no cache), 1 = per-weight cache, 2 = batched group cache
            engine.set_options(pack_cache=int(v) > 0, batch_pack=int(v) > 1)
        elif k == 'math':
            model.conv_math = v
        elif k == 'pool_diff':
            engine.set_options(pool_diff=bool(int(v)))
        elif k == 'pooled_bn_bwd':
            engine.set_options(pooled_bn_bwd=bool(int(v)))
        elif k == 'defer_bn_bwd':
            engine.set_options(defer_bn_bwd=bool(int(v)))
        elif k == 'fuse_enc':
            engine.set_options(fuse_siamese_encoder=bool(int(v)))
        elif k == 'bn_bwd_in_wgrad':  # widest weight-grad source (channels) that forms its BatchNorm backward
            engine.set_options(bn_bwd_in_wgrad=int(v))
        elif k in engine._OPTS:  # any other engine option by name (e.g. fuse_head=0)
            engine.set_options(**{k: bool(int(v))})
        else:
            raise SystemExit(f'unknown knob {k}')


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--variants', nargs='+', required=True)
    ap.add_argument('--rounds', type=int, default=6)
    ap.add_argument('--steps', type=int, default=8)
    ap.add_argument('--config', default='baseline_siamese')
    ap.add_argument('--batch', type=int, default=None)
    ap.add_argument('--math', default=None, help='cfg.MODEL.CONV_MATH (as bench.py --math; bf16 brings bf16 storage)')
    args = ap.parse_args()
    hip.load_library()
    dev = torch.device('cuda:0')
    cfg = experiment_manager.load_cfg(args.config)
    if args.math:
        cfg.MODEL.CONV_MATH = args.math
    batch = args.batch or int(cfg.TRAINER.BATCH_SIZE)
    torch.manual_seed(cfg.SEED)
    net = networks.create_network(cfg).to(dev).train()
    opt = torch.optim.AdamW(net.parameters(), lr=float(cfg.TRAINER.LR), weight_decay=0.01, fused=True)
    gen = torch.Generator(device=dev).manual_seed(7)
    b = datasets.synthetic_batch(cfg, batch, dev, gen)

    def step():  # the config's trainer loss (single-task, dual-task, MMCR: trainers.step_loss)
        opt.zero_grad(set_to_none=True)
        loss = trainers.step_loss(cfg, net(b['x_t1'], b['x_t2']), b)
        loss.backward()
        opt.step()

    times = {v: [] for v in args.variants}
    math0 = net.module.conv_math
    for v in args.variants:  # warm every variant (allocator, occupancy caches, clocks)
        apply(v, net.module, math0)
        for _ in range(3):
            step()
    torch.cuda.synchronize()
    for r in range(args.rounds):
        for v in args.variants:
            apply(v, net.module, math0)
            step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                step()
            torch.cuda.synchronize()
            times[v].append(1000.0 * (time.perf_counter() - t0) / args.steps)
    for v, ts in times.items():
        print(f'{v:30s} median {statistics.median(ts):8.3f} ms  min {min(ts):8.3f} ms  '
              f'({batch / statistics.median(ts) * 1000:.1f} pairs/s)  rounds {["%.2f" % t for t in ts]}', flush=True)


if __name__ == '__main__':
    main()
