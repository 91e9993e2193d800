"""ORACLE — TEST INFRASTRUCTURE ONLY.  Never imported by the product package.

numpy restatement of the reference's per-item augmentation chain (utils/augmentations.py:6-142) with an explicit
RandomState in place of the global np.random.  The reference module itself cannot be imported here (it needs
torchvision, absent); this follows its code line by line:

  compose_transformations   augmentations.py:6-32    crop, flip, rotate, color shift, gamma, to-tensor order
  UniformCrop.random_crop   augmentations.py:113-122 x = randint(0, W - S), then y = randint(0, H - S)
  ImportanceRandomCrop      augmentations.py:129-142 20 crops, weights = float32 label sums + 5, choice(p=w / sum)
  RandomFlip                augmentations.py:48-65   choice([True, False]) twice; np.flip axis 1, then axis 0
  RandomRotate              augmentations.py:68-74   k = randint(1, 4); np.rot90(k, axes=(0, 1))
  ColorShift                augmentations.py:77-89   uniform(0.5, 1.5, C) per image; clip(x * f, 0, 1) -> float32
  GammaCorrection           augmentations.py:92-105  uniform(0.25, 2, C); clip(x ** g, 0, 1) -> float32
  Numpy2Torch               augmentations.py:35-42   HWC -> CHW

Parity: the numpy operations are the reference's own (np.flip, np.rot90, np.clip, np.power); pinned by
construction, not by a reference run ("parity unpinned" for the module as a whole: torchvision is absent).
"""
from __future__ import annotations

import numpy as np


def chain(cfg_aug: dict, img_t1: np.ndarray, img_t2: np.ndarray, label: np.ndarray, rng):
    S = cfg_aug['CROP_SIZE']

    def random_crop(a, b, c):
        height, width, _ = c.shape
        x = rng.randint(0, width - S)
        y = rng.randint(0, height - S)
        return a[y:y + S, x:x + S], b[y:y + S, x:x + S], c[y:y + S, x:x + S]

    if cfg_aug.get('IMAGE_OVERSAMPLING_TYPE', 'none') == 'none':
        img_t1, img_t2, label = random_crop(img_t1, img_t2, label)
    else:
        crops = [random_crop(img_t1, img_t2, label) for _ in range(20)]
        w = np.array([c[2].sum() for c in crops]) + 5
        w = w / w.sum()
        img_t1, img_t2, label = crops[rng.choice(20, p=w)]
    if cfg_aug.get('RANDOM_FLIP', False):
        h = rng.choice([True, False])
        v = rng.choice([True, False])
        if h:
            img_t1, img_t2, label = np.flip(img_t1, axis=1), np.flip(img_t2, axis=1), np.flip(label, axis=1)
        if v:
            img_t1, img_t2, label = np.flip(img_t1, axis=0), np.flip(img_t2, axis=0), np.flip(label, axis=0)
        img_t1, img_t2, label = img_t1.copy(), img_t2.copy(), label.copy()
    if cfg_aug.get('RANDOM_ROTATE', False):
        k = rng.randint(1, 4)
        img_t1 = np.rot90(img_t1, k, axes=(0, 1)).copy()
        img_t2 = np.rot90(img_t2, k, axes=(0, 1)).copy()
        label = np.rot90(label, k, axes=(0, 1)).copy()
    if cfg_aug.get('COLOR_SHIFT', False):
        f1 = rng.uniform(0.5, 1.5, img_t1.shape[-1])
        img_t1 = np.clip(img_t1 * f1[np.newaxis, np.newaxis, :], 0, 1).astype(np.float32)
        f2 = rng.uniform(0.5, 1.5, img_t2.shape[-1])
        img_t2 = np.clip(img_t2 * f2[np.newaxis, np.newaxis, :], 0, 1).astype(np.float32)
    if cfg_aug.get('GAMMA_CORRECTION', False):
        g1 = rng.uniform(0.25, 2, img_t1.shape[-1])
        img_t1 = np.clip(np.power(img_t1, g1[np.newaxis, np.newaxis, :]), 0, 1).astype(np.float32)
        g2 = rng.uniform(0.25, 2, img_t2.shape[-1])
        img_t2 = np.clip(np.power(img_t2, g2[np.newaxis, np.newaxis, :]), 0, 1).astype(np.float32)
    return (np.ascontiguousarray(img_t1.transpose(2, 0, 1)), np.ascontiguousarray(img_t2.transpose(2, 0, 1)),
            np.ascontiguousarray(label.transpose(2, 0, 1)))
