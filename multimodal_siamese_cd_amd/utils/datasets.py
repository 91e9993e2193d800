"""Synthetic SAR+optical change-detection pairs with the reference's item-dict contract.

The reference's `MultimodalCDDataset` (utils/datasets.py:65-193) reads SpaceNet7 GeoTIFFs with rasterio
(not installed, no data here); that reader is out of scope.  What the training path consumes is the item
dict (datasets.py:164-179): `x_t1`, `x_t2` (C, H, W) fp32 in [0, 1], `y_change` (1, H, W) in {0, 1},
optional `y_sem_t1` / `y_sem_t2` (INCLUDE_BUILDING_LABELS) and `is_labeled`.  This module produces the same
dicts from a seeded generator, either per item (a torch Dataset for DataLoader use) or as whole batches
generated directly on the device so input generation never limits the measured step rate.
"""
from __future__ import annotations

import torch
from torch.utils.data import Dataset


def _channels(cfg) -> int:
    mode = cfg.DATALOADER.get('INPUT_MODE', 's1s2')
    n1, n2 = len(cfg.DATALOADER.S1_BANDS), len(cfg.DATALOADER.S2_BANDS)
    if mode == 's1':
        return n1
    if mode == 's2':
        return n2
    return n1 + n2


def synthetic_batch(cfg, batch_size: int, device, generator: torch.Generator, size=None,
                    change_rate: float = 0.05, sem_rate: float = 0.2):
    """One batch of item dicts stacked along dim 0, generated on `device`.  `size`: int or (H, W); default
    AUGMENTATION.CROP_SIZE (training crops); eval AOIs may be any size (networks.py:437-443 pads)."""
    c = cfg.MODEL.IN_CHANNELS if 'IN_CHANNELS' in cfg.MODEL else _channels(cfg)
    s = size or cfg.AUGMENTATION.CROP_SIZE
    h, w = (s, s) if isinstance(s, int) else tuple(s)
    kw = dict(device=device, generator=generator)
    b = {
        'x_t1': torch.rand((batch_size, c, h, w), **kw),
        'x_t2': torch.rand((batch_size, c, h, w), **kw),
        'y_change': (torch.rand((batch_size, 1, h, w), **kw) < change_rate).float(),
    }
    if cfg.DATALOADER.get('INCLUDE_BUILDING_LABELS', False) or cfg.MODEL.TYPE == 'dtsiameseunet':
        b['y_sem_t1'] = (torch.rand((batch_size, 1, h, w), **kw) < sem_rate).float()
        b['y_sem_t2'] = (torch.rand((batch_size, 1, h, w), **kw) < sem_rate).float()
    frac = float(cfg.DATALOADER.get('LABELED_FRACTION', 1.0))
    n_lab = max(1, int(round(frac * batch_size))) if frac > 0 else 0
    b['is_labeled'] = torch.arange(batch_size, device=device) < n_lab
    return b


class SyntheticCDDataset(Dataset):
    """Per-item synthetic dataset (CPU tensors), deterministic in (seed, index)."""

    def __init__(self, cfg, run_type: str = 'training', length: int | None = None, seed: int | None = None,
                 size=None):
        self.cfg = cfg
        self.run_type = run_type
        self.size = size
        self.length = length if length is not None else int(cfg.TRAINER.get('STEPS_PER_EPOCH', 100)) * int(
            cfg.TRAINER.BATCH_SIZE)
        self.seed = int(cfg.SEED if seed is None else seed)

    def __len__(self):
        return self.length

    def __getitem__(self, index):
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + index)
        item = synthetic_batch(self.cfg, 1, 'cpu', g, size=self.size)
        out = {k: v[0] for k, v in item.items()}
        out['is_labeled'] = bool(index % 2 == 0) if self.cfg.DATALOADER.get('INCLUDE_UNLABELED', False) else True
        out['aoi_id'] = f'synthetic_{index:06d}'
        return out

    def __str__(self):
        return f'Dataset with {self.length} samples.'
