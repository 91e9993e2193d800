"""Training augmentations — the reference's utils/augmentations.py:6-142, applied to a whole batch on the device.

The reference composes per-item numpy transforms in DataLoader workers (compose_transformations,
augmentations.py:6-32).  Here the random parameters are drawn on the host in exactly the reference's per-item
order (so a seeded numpy RandomState gives the reference's draws), and the pixel work of every item runs in two
HIP launches per channel group:

  ImportanceRandomCrop  augmentations.py:129-142  20 uniform candidates; their change-label sums on the device
                                                   (scd_window_label_sums); weight = sum + 5; np.random.choice
  UniformCrop           augmentations.py:108-126
  RandomFlip            augmentations.py:48-65    horizontal (axis 1), then vertical (axis 0)
  RandomRotate          augmentations.py:68-74    k in {1, 2, 3} quarter turns, axes (0, 1)
  ColorShift            augmentations.py:77-89    factors U(0.5, 1.5) per channel, clip to [0, 1]
  GammaCorrection       augmentations.py:92-105   gammas U(0.25, 2) per channel, clip to [0, 1]
  Numpy2Torch           augmentations.py:35-42    HWC -> CHW

As in the reference, the chain receives (imgs, buildings, change) as (img_t1, img_t2, label) (datasets.py:165):
ColorShift / GammaCorrection use the "t1" draws on all image bands and the "t2" draws on the two building-label
channels, and crops are weighted by the change label.
"""
from __future__ import annotations

import numpy as np
import torch

from .. import hip

IMPORTANCE_SAMPLES = 20    # augmentations.py:132
IMPORTANCE_BALANCE = 5     # augmentations.py:133


class _Params:
    """Per-item random parameters, drawn in the reference's call order."""

    def __init__(self):
        self.candidates = None  # [(y, x)] for ImportanceRandomCrop, else one (y, x)
        self.u = None           # the uniform sample np.random.choice(p=...) draws
        self.flip_h = self.flip_v = False
        self.rot = 0
        self.scale = None       # (factors_t1 [C_img], factors_t2 [2])
        self.gamma = None


class DeviceAugmentation:
    """compose_transformations(cfg, no_augmentations) as one batched device transform."""

    def __init__(self, cfg, no_augmentations: bool):
        a = cfg.AUGMENTATION
        self.crop = int(a.CROP_SIZE)
        self.no_augmentations = no_augmentations
        self.importance = a.get('IMAGE_OVERSAMPLING_TYPE', 'none') != 'none'
        self.flip = bool(a.get('RANDOM_FLIP', False))
        self.rotate = bool(a.get('RANDOM_ROTATE', False))
        self.color = bool(a.get('COLOR_SHIFT', False))
        self.gamma = bool(a.get('GAMMA_CORRECTION', False))

    def draw(self, rng, height: int, width: int, n_img: int, n_t2: int) -> _Params:
        """One item's draws (augmentations.py:113-142, 48-105) from a numpy RandomState / np.random."""
        p = _Params()
        lim_x, lim_y = width - self.crop, height - self.crop

        def crop():
            x = rng.randint(0, lim_x)  # x first, then y (augmentations.py:117-118)
            y = rng.randint(0, lim_y)
            return y, x

        if self.importance:
            p.candidates = [crop() for _ in range(IMPORTANCE_SAMPLES)]
            p.u = rng.random_sample()  # what np.random.choice(n, p=w) consumes
        else:
            p.candidates = [crop()]
        if self.flip:
            p.flip_h = bool(rng.choice([True, False]))
            p.flip_v = bool(rng.choice([True, False]))
        if self.rotate:
            p.rot = int(rng.randint(1, 4))
        if self.color:
            p.scale = (rng.uniform(0.5, 1.5, n_img), rng.uniform(0.5, 1.5, n_t2))
        if self.gamma:
            p.gamma = (rng.uniform(0.25, 2, n_img), rng.uniform(0.25, 2, n_t2))
        return p

    def __call__(self, imgs: list, buildings: list, change: list, draws=None, rng=np.random):
        """Per-item device HWC tiles -> (imgs [B, C, S, S], buildings [B, 2, S, S], change [B, 1, S, S]).
        `draws`: per-item parameters drawn earlier (the dataset draws them in __getitem__, interleaved with its own
        draws as the reference's per-item transform is); None = draw them now from `rng`."""
        if self.no_augmentations:  # Numpy2Torch only: full tiles, one item at a time in the reference
            return (torch.stack([t.permute(2, 0, 1) for t in imgs]), torch.stack([t.permute(2, 0, 1) for t in buildings]),
                    torch.stack([t.permute(2, 0, 1) for t in change]))
        S = self.crop
        if draws is None:
            draws = [self.draw(rng, t.shape[0], t.shape[1], imgs[0].shape[2], buildings[0].shape[2]) for t in change]
        chosen = [d.candidates[0] for d in draws]
        if self.importance:
            yx = torch.tensor([d.candidates for d in draws], dtype=torch.int32)
            sums = hip.window_label_sums([c.reshape(c.shape[0], c.shape[1]) for c in change], yx, S).cpu().numpy()
            for b, d in enumerate(draws):
                w = sums[b].astype(np.float32) + IMPORTANCE_BALANCE  # float32 label sums + 5, as the reference
                w = w / w.sum()
                cdf = w.astype(np.float64).cumsum()  # RandomState.choice(p=...): float64 cdf, one random_sample
                cdf /= cdf[-1]
                chosen[b] = d.candidates[int(cdf.searchsorted(d.u, side='right'))]
        params = torch.tensor([[y, x, int(d.flip_h), int(d.flip_v), d.rot] for (y, x), d in zip(chosen, draws)],
                              dtype=torch.int32)

        def per_group(i):
            sc = torch.tensor(np.stack([d.scale[i] for d in draws])) if self.color else None
            gm = torch.tensor(np.stack([d.gamma[i] for d in draws])) if self.gamma else None
            return sc, gm

        s1, g1 = per_group(0)
        s2, g2 = per_group(1)
        out_imgs = hip.augment_apply(imgs, S, params, s1, g1)
        out_bld = hip.augment_apply(buildings, S, params, s2, g2)
        out_chg = hip.augment_apply(change, S, params)
        return out_imgs, out_bld, out_chg


def compose_transformations(cfg, no_augmentations: bool) -> DeviceAugmentation:
    return DeviceAugmentation(cfg, no_augmentations)
