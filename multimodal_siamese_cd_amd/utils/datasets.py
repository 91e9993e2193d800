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


def uses_synthetic_data(cfg) -> bool:
    """Whether a run trains/evaluates on synthetic pairs rather than the tile cache.

    DATALOADER.SYNTHETIC unset (None, the shipped default) means: synthetic exactly when the config names no
    training AOIs, so a reference config that carries its DATASET.*_IDS split reads real tiles.  An explicit
    True next to a non-empty split is honoured, with a loud warning.
    """
    flag = cfg.DATALOADER.get('SYNTHETIC', None)
    ids = list(cfg.get('DATASET', {}).get('TRAINING_IDS', []) or [])
    if flag is None:
        return not ids
    if flag and ids:
        import warnings
        warnings.warn(f'DATALOADER.SYNTHETIC is True although DATASET.TRAINING_IDS names {len(ids)} AOIs: '
                      'training on synthetic noise, not on the tile cache', stacklevel=2)
    return bool(flag)


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


# ------------------------------------------------------------------------------------------------
# SpaceNet7 multimodal change-detection dataset over an offline tile cache
# ------------------------------------------------------------------------------------------------
class MultimodalCDDataset(Dataset):
    """utils/datasets.py:9-193 (AbstractMultimodalCDDataset + MultimodalCDDataset) with the same constructor,
    AOI selection, labelled/unlabelled lists, timestamp choice and item contract.

    Differences, by design:
      - tiles come from an offline cache with the reference's directory layout, `.npy` (H, W, C) float32 in place
        of the GeoTIFFs (rasterio is not available): <root>/<aoi>/s1/s1_<aoi>_<year>_<mm>.npy, likewise s2 and
        buildings, plus the reference's metadata.json;
      - __getitem__ returns the raw full tiles and the augmentation draws (made here, after this item's own
        timestamp draws, in the reference's order); `device_collate` runs the transform chain for a whole batch
        on the GPU (utils/augmentations.py).  No multiprocessing.Manager proxies (datasets.py:103-107).
    """

    def __init__(self, cfg, run_type: str, no_augmentations: bool = False, dataset_mode: str = None,
                 disable_multiplier: bool = False, disable_unlabeled: bool = False, rng=None):
        import json
        from pathlib import Path

        import numpy as np

        from . import augmentations
        self.cfg = cfg
        self.run_type = run_type
        self.root_path = Path(cfg.PATHS.DATASET)
        with open(self.root_path / 'metadata.json') as f:
            self.metadata = json.load(f)
        self.s1_band_indices = list(cfg.DATALOADER.S1_BANDS)
        self.s2_band_indices = list(cfg.DATALOADER.S2_BANDS)
        self.rng = np.random if rng is None else rng
        self.dataset_mode = cfg.DATALOADER.DATASET_MODE if dataset_mode is None else dataset_mode
        self.include_building_labels = bool(cfg.DATALOADER.get('INCLUDE_BUILDING_LABELS', False))
        self.no_augmentations = no_augmentations
        self.transform = augmentations.compose_transformations(cfg, no_augmentations)
        ids = {'training': 'TRAINING_IDS', 'validation': 'VALIDATION_IDS'}.get(run_type, 'TEST_IDS')
        self.aoi_ids = list(cfg.DATASET[ids])
        self.labeled = [True] * len(self.aoi_ids)
        dl = cfg.DATALOADER
        if (dl.get('INCLUDE_UNLABELED', False) or dl.get('INCLUDE_UNLABELED_VALIDATION', False)) and not disable_unlabeled:
            unl = []
            if dl.get('INCLUDE_UNLABELED', False):
                unl += list(cfg.DATASET.UNLABELED_IDS)
            if dl.get('INCLUDE_UNLABELED_VALIDATION', False):
                unl += list(cfg.DATASET.VALIDATION_IDS)
            unl = sorted(unl)
            self.aoi_ids.extend(unl)
            self.labeled.extend([False] * len(unl))
        if not disable_multiplier:
            mult = int(dl.get('TRAINING_MULTIPLIER', 1))
            self.aoi_ids = self.aoi_ids * mult
            self.labeled = self.labeled * mult
        self.length = len(self.aoi_ids)

    # loaders (datasets.py:30-52): band selection, clip to [0, 1], NaN -> 0
    def _npy(self, aoi_id, kind, year, month):
        import numpy as np
        return np.load(self.root_path / aoi_id / kind / f'{kind}_{aoi_id}_{year}_{month:02d}.npy')

    def _load_s1_img(self, aoi_id, year, month):
        import numpy as np
        img = np.clip(self._npy(aoi_id, 's1', year, month)[:, :, self.s1_band_indices], 0, 1)
        return np.nan_to_num(img).astype(np.float32)

    def _load_s2_img(self, aoi_id, year, month):
        import numpy as np
        img = np.clip(self._npy(aoi_id, 's2', year, month)[:, :, self.s2_band_indices], 0, 1)
        return np.nan_to_num(img).astype(np.float32)

    def _load_building_label(self, aoi_id, year, month):
        import numpy as np
        return np.nan_to_num(self._npy(aoi_id, 'buildings', year, month) > 0).astype(np.float32)

    def _load_change_label(self, aoi_id, year_t1, month_t1, year_t2, month_t2):
        import numpy as np
        b1 = self._load_building_label(aoi_id, year_t1, month_t1)
        b2 = self._load_building_label(aoi_id, year_t2, month_t2)
        return np.logical_and(b1 == 0, b2 == 1).astype(np.float32)

    def __getitem__(self, index):
        import numpy as np
        aoi_id = self.aoi_ids[index]
        labeled = self.labeled[index]
        ts = self.metadata[aoi_id]
        if labeled:
            ts = [(t['year'], t['month']) for t in ts if t['s1'] and t['s2'] and t['buildings'] and not t['masked']]
        else:
            ts = [(t['year'], t['month']) for t in ts if t['s1'] and t['s2']]
        idx = [0, -1] if self.dataset_mode == 'first_last' else sorted(self.rng.randint(0, len(ts), size=2))
        (y1, m1), (y2, m2) = ts[idx[0]], ts[idx[1]]
        s1_t1, s2_t1 = self._load_s1_img(aoi_id, y1, m1), self._load_s2_img(aoi_id, y1, m1)
        s1_t2, s2_t2 = self._load_s1_img(aoi_id, y2, m2), self._load_s2_img(aoi_id, y2, m2)
        if labeled:
            change = self._load_change_label(aoi_id, y1, m1, y2, m2)
            if self.include_building_labels:
                buildings = np.concatenate((self._load_building_label(aoi_id, y1, m1),
                                            self._load_building_label(aoi_id, y2, m2)), axis=-1).astype(np.float32)
            else:
                buildings = np.zeros((change.shape[0], change.shape[1], 2), dtype=np.float32)
        else:
            change = np.zeros((s1_t1.shape[0], s1_t1.shape[1], 1), dtype=np.float32)
            buildings = np.zeros((change.shape[0], change.shape[1], 2), dtype=np.float32)
        imgs = np.concatenate((s1_t1, s1_t2, s2_t1, s2_t2), axis=-1)
        draws = None
        if not self.no_augmentations:
            draws = self.transform.draw(self.rng, change.shape[0], change.shape[1], imgs.shape[2], buildings.shape[2])
        return {'imgs': imgs, 'buildings': buildings, 'change': change, 'aug': draws, 'aoi_id': aoi_id,
                'year_t1': y1, 'month_t1': m1, 'year_t2': y2, 'month_t2': m2, 'is_labeled': labeled}

    def get_index(self, aoi_id: str):
        for index, candidate in enumerate(self.aoi_ids):
            if aoi_id == candidate:
                return index
        return None

    def get_aoi_ids(self) -> list:
        return list(set(self.aoi_ids))

    def __len__(self):
        return self.length

    def __str__(self):
        return f'Dataset with {self.length} samples.'


def device_collate(items: list, dataset: MultimodalCDDataset, device) -> dict:
    """Raw items -> the reference's batched item dict (datasets.py:164-179) with the transforms of
    utils/augmentations.py run on the device for the whole batch."""
    import numpy as np
    up = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)
    imgs, bld, chg = dataset.transform([up(it['imgs']) for it in items], [up(it['buildings']) for it in items],
                                       [up(it['change']) for it in items], draws=[it['aug'] for it in items])
    n1, n2 = len(dataset.s1_band_indices), len(dataset.s2_band_indices)
    s1_t1, s1_t2 = imgs[:, :n1], imgs[:, n1:2 * n1]
    s2_t1, s2_t2 = imgs[:, 2 * n1:2 * n1 + n2], imgs[:, 2 * n1 + n2:]
    mode = dataset.cfg.DATALOADER.get('INPUT_MODE', 's1s2')
    if mode == 's1':
        x_t1, x_t2 = s1_t1, s1_t2
    elif mode == 's2':
        x_t1, x_t2 = s2_t1, s2_t2
    else:
        x_t1, x_t2 = torch.cat((s1_t1, s2_t1), 1), torch.cat((s1_t2, s2_t2), 1)
    out = {'x_t1': x_t1.contiguous(), 'x_t2': x_t2.contiguous(), 'y_change': chg,
           'is_labeled': torch.tensor([it['is_labeled'] for it in items], device=device)}
    for k in ('aoi_id', 'year_t1', 'month_t1', 'year_t2', 'month_t2'):
        out[k] = [it[k] for it in items]
    if dataset.include_building_labels:
        out['y_sem_t1'] = bld[:, 0:1].contiguous()
        out['y_sem_t2'] = bld[:, 1:2].contiguous()
    return out


class DeviceDataLoader:
    """DataLoader over MultimodalCDDataset whose workers only read tiles; batches are augmented on the device."""

    def __init__(self, dataset: MultimodalCDDataset, batch_size: int, device, shuffle: bool = True,
                 drop_last: bool = True, num_workers: int = 0, distributed: bool = True):
        """`distributed=False` never shards: the evaluation path scores the whole split on one rank."""
        import torch.distributed as dist
        from torch.utils.data import DataLoader, DistributedSampler
        self.dataset, self.device = dataset, device
        sampler = None
        if distributed and dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            # one shard per rank (training)
            sampler = DistributedSampler(dataset, shuffle=shuffle, drop_last=drop_last)
            shuffle = False
        self.sampler = sampler
        self.loader = DataLoader(dataset, batch_size=batch_size, shuffle=shuffle, drop_last=drop_last,
                                 num_workers=num_workers, collate_fn=list, sampler=sampler)

    def set_epoch(self, epoch: int):
        if self.sampler is not None:
            self.sampler.set_epoch(epoch)

    def __len__(self):
        return len(self.loader)

    def __iter__(self):
        for items in self.loader:
            yield device_collate(items, self.dataset, self.device)
