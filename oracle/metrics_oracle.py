"""ORACLE — TEST INFRASTRUCTURE ONLY.  Never imported by the product package.

numpy restatement of the reference's MultiThresholdMetric counting (utils/metrics.py:22-31):

  y_true.bool()                               -> label = y != 0 (NaN is True)            metrics.py:23
  (y_pred - thr + 0.5).round().bool()         -> v = (p - t) + 0.5 in float32 (two roundings);
                                                 round half to even is 0 exactly when -0.5 <= v <= 0.5,
                                                 so positive = not (-0.5 <= v <= 0.5) (NaN positive)  metrics.py:26
  TP = label & pos, TN = ~label & ~pos, FP = label & ~pos, FN = ~label & pos (the reference's naming)
                                                                                         metrics.py:28-31

Pinned against tests/golden/metrics_mt.npz (made by running utils/metrics.py itself) in
tests/test_eval_path.py.  Also restates the F.pad window of Up.forward (networks.py:437-443) for the window-copy
kernel test.
"""
from __future__ import annotations

import numpy as np


def positive(p: np.ndarray, thr: float) -> np.ndarray:
    p = np.asarray(p, dtype=np.float32)
    with np.errstate(invalid='ignore'):
        v = (p - np.float32(thr)).astype(np.float32) + np.float32(0.5)
        return ~((v >= np.float32(-0.5)) & (v <= np.float32(0.5)))


def confusion(y_true: np.ndarray, y_pred: np.ndarray, thresholds) -> dict:
    """int64 TP, TN, FP, FN per threshold (reference naming)."""
    with np.errstate(invalid='ignore'):
        lab = np.asarray(y_true, dtype=np.float32) != 0
        lab = lab | np.isnan(np.asarray(y_true, dtype=np.float32))
    out = {k: [] for k in ('TP', 'TN', 'FP', 'FN')}
    for t in np.asarray(thresholds, dtype=np.float32).reshape(-1):
        pos = positive(y_pred, t)
        out['TP'].append(np.sum(lab & pos))
        out['TN'].append(np.sum(~lab & ~pos))
        out['FP'].append(np.sum(lab & ~pos))
        out['FN'].append(np.sum(~lab & pos))
    return {k: np.array(v, dtype=np.int64) for k, v in out.items()}


def kernel_counts(y_true: np.ndarray, y_pred: np.ndarray, thresholds) -> np.ndarray:
    """The layout scd_threshold_counts returns: {#label, then per threshold: TP, #positive}."""
    c = confusion(y_true, y_pred, thresholds)
    n_true = int(c['TP'][0] + c['FP'][0])
    out = [n_true]
    for k in range(len(c['TP'])):
        out += [int(c['TP'][k]), int(c['TP'][k] + c['FN'][k])]
    return np.array(out, dtype=np.int64)


def pad_window(up: np.ndarray, h: int, w: int) -> np.ndarray:
    """F.pad(x1, (dX//2, dX - dX//2, dY//2, dY - dY//2)) of an NHWC map to (h, w) (networks.py:437-443)."""
    n, hu, wu, c = up.shape
    dy, dx = h - hu, w - wu
    out = np.zeros((n, h, w, c), dtype=up.dtype)
    out[:, dy // 2:dy // 2 + hu, dx // 2:dx // 2 + wu] = up
    return out
