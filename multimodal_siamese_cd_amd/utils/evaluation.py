"""Eval path — drop-in for the reference's utils/evaluation.py:7-41 (`model_evaluation`).

Same loop as the reference: net.eval(), batch size 1 over the run's AOIs (full tiles of any size: the decoder's
Up zero-pads when a size is not divisible by 2**levels, networks.py:437-443), thresholds linspace(0.5, 1, 1),
F1 / precision / recall at the best threshold.  Differences, by design:
  - the sigmoid and the thresholded confusion counts run as one fused HIP pass (MultiThresholdMetric.add_logits,
    `scd_threshold_counts`) instead of sigmoid + 4 boolean reductions;
  - wandb is not installed: the numbers go to `log` (default print) and are returned as a dict;
  - with real data (datasets.uses_synthetic_data False) the run's AOIs come from the tile cache (datasets.MultimodalCDDataset, as
    evaluation.py:15-17 builds it); otherwise `dataset` defaults to the synthetic item-dict dataset.
  - a model returning a tuple (DualTaskSiameseUNet) is scored on its change output (index 0); the reference
    would fail on it.
"""
from __future__ import annotations

import torch
from torch.utils import data as torch_data

from . import datasets, metrics


def model_evaluation(net, cfg, device, run_type: str, epoch: float, step: int, dataset=None, log=None,
                     thresholds=None) -> dict:
    net.to(device)
    net.eval()
    thr = torch.linspace(0.5, 1, 1) if thresholds is None else torch.as_tensor(thresholds, dtype=torch.float32)
    measurer = metrics.MultiThresholdMetric(thr)
    if dataset is None and not datasets.uses_synthetic_data(cfg):  # evaluation.py:15-17
        dataset = datasets.MultimodalCDDataset(cfg, run_type, no_augmentations=True, dataset_mode='first_last',
                                               disable_multiplier=True, disable_unlabeled=True)
    ds = dataset if dataset is not None else datasets.SyntheticCDDataset(
        cfg, run_type, length=int(cfg.get('EVAL_SAMPLES', 4)), seed=int(cfg.SEED) + 1000)
    if isinstance(ds, datasets.MultimodalCDDataset):  # full tiles, transforms (to-tensor only) on the device
        # distributed=False: evaluation runs on rank 0 only and must see every AOI of the split, unpadded
        dataloader = datasets.DeviceDataLoader(ds, 1, device, shuffle=False, drop_last=False, distributed=False)
    else:
        dataloader = torch_data.DataLoader(ds, batch_size=1, num_workers=0, shuffle=False, drop_last=False)
    with torch.no_grad():
        for item in dataloader:
            x_t1 = item['x_t1'].to(device)
            x_t2 = item['x_t2'].to(device)
            logits = net(x_t1, x_t2)
            if isinstance(logits, (tuple, list)):
                logits = logits[0]
            gt = item['y_change'].to(device)
            measurer.add_logits(gt, logits)

    f1s = measurer.compute_f1()
    precisions, recalls = measurer.precision, measurer.recall
    f1 = f1s.max().item()
    argmax_f1 = f1s.argmax()
    out = {
        f'{run_type} F1': f1,
        f'{run_type} precision': precisions[argmax_f1].item(),
        f'{run_type} recall': recalls[argmax_f1].item(),
        'step': step, 'epoch': epoch,
    }
    (log or print)(out)
    return out
