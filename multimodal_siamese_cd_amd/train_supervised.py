"""Training entry point — counterpart of the reference's train_supervised.py (also covers the dual-task and
MMCR trainers' per-step losses, train_supervised_dualtask.py / train_semisupervised.py).

    python -m multimodal_siamese_cd_amd.train_supervised -c baseline_siamese -p proj -o out/ -d data/ [KEY VALUE ...]
    torchrun --nproc-per-node 8 -m multimodal_siamese_cd_amd.train_supervised -c baseline_dualstream ...

Step loop (train_supervised.py:63-79): net.train(); zero_grad; forward; loss; backward; AdamW(lr, wd=0.01).
Differences, by design: data are synthetic pairs generated on the device (the SpaceNet7 GeoTIFF reader is out
of scope), wandb logging is replaced by stdout, the per-step `loss.item()` host sync happens only every
LOG_FREQ steps, and multi-GPU is one process per GPU (DDP over RCCL) instead of nn.DataParallel.
"""
from __future__ import annotations

import sys
import timeit

import numpy as np
import torch

from . import engine, hip, parallel, trainers  # noqa: F401
from .utils import datasets, evaluation, experiment_manager, networks, parsers


def _evaluate(net, cfg, device, run_types, epoch_float, step, rank):
    """evaluation.model_evaluation on rank 0 (the reference evaluates its single DataParallel process,
    train_supervised.py:84-113), on the unwrapped module so no DDP collective is involved; back to train mode."""
    if rank != 0 or not cfg.get('EVALUATE', True):
        return
    module = net.module if isinstance(net, torch.nn.parallel.DistributedDataParallel) else net
    for rt in run_types:
        evaluation.model_evaluation(module, cfg, device, rt, epoch_float, step)
    net.train()


def _checked_loss(value: float, cfg, step: int) -> float:
    """The logged loss (a host sync the loop makes anyway), refused when non-finite.  Under MODEL.PRECISION fp32 the
    convs run h2 (engine.conv_math_for), whose operand scaling relies on every producer's magnitude bound: an
    underestimated bound overflows fp16 into inf / NaN, so the error names the arithmetic that was active."""
    if not np.isfinite(value):
        raise FloatingPointError(f"non-finite training loss {value} at step {step} (conv arithmetic "
                                 f"{engine.conv_math_for(cfg)!r}; MODEL.CONV_MATH x3 is the bound-free fp32-class "
                                 "alternative)")
    return value


def _check_finite(bad, cfg, first: int, step: int, device) -> None:
    """Raise on every rank when any of the steps first..step (those since the last check) produced a non-finite loss on
    any rank: the flag is max-all-reduced, so no rank is left waiting in a DDP collective while another one stops."""
    flag = torch.zeros(1, device=device) if bad is None else bad.float().reshape(1)
    if parallel.is_distributed():
        torch.distributed.all_reduce(flag, op=torch.distributed.ReduceOp.MAX)
    if flag.item() > 0:
        raise FloatingPointError(f"non-finite training loss within steps {first}..{step} "
                                 f"(conv arithmetic {engine.conv_math_for(cfg)!r}; MODEL.CONV_MATH x3 is the bound-free "
                                 "fp32-class alternative)")


def run_training(cfg, device, max_steps: int | None = None):
    rank, _, world = parallel.env_rank()
    net = networks.create_network(cfg)
    net.to(device)
    # TRAINER.EXACT_DATAPARALLEL: the reference's gathered-batch loss of nn.DataParallel (one loss over all ranks'
    # pairs, summed gradients) instead of DDP's mean of per-rank losses (parallel.wrap_ddp)
    net = parallel.wrap_ddp(net, device, exact_dataparallel=bool(cfg.TRAINER.get('EXACT_DATAPARALLEL', False)))
    optimizer = torch.optim.AdamW(net.parameters(), lr=float(cfg.TRAINER.LR), weight_decay=0.01)
    gen = torch.Generator(device=device).manual_seed(parallel.rank_seed(cfg.SEED, rank))
    steps_per_epoch = int(cfg.TRAINER.get('STEPS_PER_EPOCH', 100))
    epochs = int(cfg.TRAINER.EPOCHS)
    global_step = 0
    if rank == 0:
        print(f"run config {cfg.NAME}: model {cfg.MODEL.TYPE} topology {list(cfg.MODEL.TOPOLOGY)} "
              f"bs {cfg.TRAINER.BATCH_SIZE}/GPU x {world} GPU, lr {cfg.TRAINER.LR}, epochs {epochs}", flush=True)
    loader = None
    if not datasets.uses_synthetic_data(cfg):  # SpaceNet7 tile cache, augmented on the device
        ds = datasets.MultimodalCDDataset(cfg, 'training')
        loader = datasets.DeviceDataLoader(ds, int(cfg.TRAINER.BATCH_SIZE), device, shuffle=bool(cfg.DATALOADER.SHUFFLE),
                                           num_workers=int(cfg.DATALOADER.get('NUM_WORKER', 0)))
        steps_per_epoch = len(loader)
    bad = None
    first_unchecked = 1  # the first step the next _check_finite covers
    for epoch in range(1, epochs + 1):
        start = timeit.default_timer()
        losses = []
        if loader is not None:
            loader.set_epoch(epoch)
        batches = iter(loader) if loader is not None else None
        for _ in range(steps_per_epoch):
            batch = next(batches) if batches is not None else datasets.synthetic_batch(
                cfg, int(cfg.TRAINER.BATCH_SIZE), device, gen)
            net.train()
            optimizer.zero_grad(set_to_none=True)
            out = net(batch['x_t1'], batch['x_t2'])
            loss = trainers.step_loss(cfg, out, batch, net)
            loss.backward()
            optimizer.step()
            losses.append(loss.detach())
            # device-side non-finite flag of every step (no host sync); checked on every rank at the log step
            bad = ~torch.isfinite(loss.detach()) if bad is None else bad | ~torch.isfinite(loss.detach())
            global_step += 1
            epoch_float = global_step / steps_per_epoch
            if cfg.DEBUG:
                _evaluate(net, cfg, device, ('test',), epoch_float, global_step, rank)
                break
            if global_step % int(cfg.LOG_FREQ) == 0:
                _check_finite(bad, cfg, first_unchecked, global_step, device)  # every rank raises together
                bad, first_unchecked = None, global_step + 1
            if global_step % int(cfg.LOG_FREQ) == 0 and rank == 0:
                t = timeit.default_timer() - start
                mean_loss = _checked_loss(torch.stack(losses).mean().item(), cfg, global_step)
                print(f'step {global_step} epoch {epoch_float:.2f} loss {mean_loss:.5f} time {t:.1f}s', flush=True)
                _evaluate(net, cfg, device, ('training', 'validation'), epoch_float, global_step, rank)
            if max_steps is not None and global_step >= max_steps:
                break
        # every rank checks the steps since the last log-step check (the epoch's tail when steps_per_epoch is not a
        # multiple of LOG_FREQ, a DEBUG or max_steps break) before rank 0 reports the epoch: a non-finite loss there
        # stops every rank together instead of rank 0 alone while the others enter the next collective
        if global_step >= first_unchecked:
            _check_finite(bad, cfg, first_unchecked, global_step, device)
        bad, first_unchecked = None, global_step + 1
        if not cfg.DEBUG:  # evaluation at the end of an epoch (train_supervised.py:107-110)
            _evaluate(net, cfg, device, ('training', 'validation', 'test'), global_step / steps_per_epoch,
                      global_step, rank)
        if rank == 0:
            print(f'epoch {epoch}: mean loss {_checked_loss(torch.stack(losses).mean().item(), cfg, global_step):.5f}',
                  flush=True)
            if epoch in list(cfg.SAVE_CHECKPOINTS) and not cfg.DEBUG:
                networks.save_checkpoint(net, optimizer, epoch, global_step, cfg)
        if cfg.DEBUG or (max_steps is not None and global_step >= max_steps):
            break
    return net, optimizer, global_step


def main(argv=None):
    args = parsers.training_argument_parser().parse_known_args(argv)[0]
    cfg = experiment_manager.setup_cfg(args)
    torch.manual_seed(cfg.SEED)
    np.random.seed(cfg.SEED)
    rank, local_rank, world = parallel.init_distributed()
    if not torch.cuda.is_available():
        raise SystemExit('train_supervised: needs an MI355X (gfx950) GPU; the HIP path has no CPU fallback')
    device = torch.device('cuda', parallel.device_index(local_rank))
    torch.cuda.set_device(device)
    hip.load_library()
    try:
        run_training(cfg, device)
    except KeyboardInterrupt:
        sys.exit(0)
    finally:
        if parallel.is_distributed():
            torch.distributed.destroy_process_group()


if __name__ == '__main__':
    main()
