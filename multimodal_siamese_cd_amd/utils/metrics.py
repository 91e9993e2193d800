"""Change-detection metrics — drop-in for the reference's utils/metrics.py.

`MultiThresholdMetric` (metrics.py:5-59) keeps the reference's API and float32 running totals (TP, TN, FP, FN;
note the reference's naming: FP = label & ~prediction, FN = ~label & prediction, metrics.py:28-31).  Its
`add_sample` is one fused HIP pass, `scd_threshold_counts`: a thresholded confusion count for up to 16
thresholds per launch, which reads the probability (or, via `add_logits`, the logit with the sigmoid of
utils/evaluation.py:25 folded in) and the label once.  The kernel returns exact integer counts; the float32
accumulation below then adds them in the reference's order (metrics.py:28-31), so the totals are bit-identical
to the reference's for the same inputs.

The small functional helpers (metrics.py:62-145) operate on whole tensors as in the reference; they are not on
the training or eval hot path.
"""
from __future__ import annotations

import numpy as np
import torch

from .. import hip

_CLAMP = 10e-05  # the reference's clamp floor (metrics.py:41, 52, 71)


def confusion_from_counts(counts: torch.Tensor, n: int):
    """(TP, TN, FP, FN) int64 per threshold, in the reference's naming, from scd_threshold_counts' output
    {#label, then per threshold: #(label & positive), #positive}."""
    counts = counts.to(torch.int64)
    n_true = counts[0]
    tp = counts[1::2]
    n_pos = counts[2::2]
    fp = n_true - tp           # label & ~prediction   (metrics.py:30)
    fn = n_pos - tp            # ~label & prediction   (metrics.py:31)
    tn = n - n_true - n_pos + tp
    return tp, tn, fp, fn


class MultiThresholdMetric(object):
    """utils/metrics.py:5-59: confusion totals over a vector of thresholds, accumulated over samples."""

    def __init__(self, threshold):
        threshold = torch.as_tensor(threshold, dtype=torch.float32)
        self._threshold_vec = threshold.reshape(-1).contiguous()
        self._thresholds = threshold[:, None, None, None, None]  # [Thresh, B, C, H, W] (metrics.py:8)
        self._data_dims = (-1, -2, -3, -4)
        self.TP = 0
        self.TN = 0
        self.FP = 0
        self.FN = 0

    def _counts(self, y_true: torch.Tensor, y_pred: torch.Tensor, from_logits: bool) -> torch.Tensor:
        hip.ensure_device(y_pred)
        pred = y_pred.detach().float().contiguous()
        truth = y_true.detach().to(device=pred.device, dtype=torch.float32).contiguous()
        if truth.numel() != pred.numel():
            raise ValueError(f"add_sample: {truth.numel()} labels vs {pred.numel()} predictions")
        thr = self._threshold_vec.to(pred.device)
        T = thr.numel()
        n = pred.numel()
        parts = []
        for k0 in range(0, T, hip.THRESHOLD_MAX):
            tk = thr[k0:k0 + hip.THRESHOLD_MAX].contiguous()
            c = torch.empty(1 + 2 * tk.numel(), dtype=torch.int64, device=pred.device)
            ws = torch.empty(hip.threshold_counts_workspace_bytes(n, tk.numel()), dtype=torch.uint8,
                             device=pred.device)
            hip.threshold_counts(pred, truth, tk, from_logits, c, ws)
            parts.append(c if k0 == 0 else c[1:])
        return torch.cat(parts) if len(parts) > 1 else parts[0]

    def _accumulate(self, counts: torch.Tensor, n: int):
        tp, tn, fp, fn = confusion_from_counts(counts, n)
        # metrics.py:28-31: int64 per-sample sums -> .float() -> float32 running totals
        self.TP += tp.float()
        self.TN += tn.float()
        self.FP += fp.float()
        self.FN += fn.float()
        for attr in ('_precision', '_recall'):
            if hasattr(self, attr):
                delattr(self, attr)

    def add_sample(self, y_true: torch.Tensor, y_pred: torch.Tensor):
        """y_pred: probabilities (metrics.py:22), on the HIP device."""
        self._accumulate(self._counts(y_true, y_pred, False), y_pred.numel())

    def add_logits(self, y_true: torch.Tensor, logits: torch.Tensor):
        """add_sample(y_true, sigmoid(logits)) with the sigmoid fused into the counting pass (evaluation.py:25).

        Bit-exact against the reference except for a pixel whose probability lies within 2 fp32 ulp of a
        threshold: there the device's 1/(1+expf(-x)) and the CPU torch.sigmoid can round to neighbouring floats
        and flip that pixel's decision (tests/test_eval_path.py::test_threshold_counts_from_logits bounds the
        count difference by that band).  `add_sample` on probabilities is bit-exact everywhere."""
        self._accumulate(self._counts(y_true, logits, True), logits.numel())

    @property
    def precision(self):
        if hasattr(self, '_precision'):
            return self._precision
        denom = (self.TP + self.FP).clamp(_CLAMP)
        self._precision = self.TP / denom
        return self._precision

    @property
    def recall(self):
        if hasattr(self, '_recall'):
            return self._recall
        denom = (self.TP + self.FN).clamp(_CLAMP)
        self._recall = self.TP / denom
        return self._recall

    def compute_basic_metrics(self):
        """(false positive rate, false negative rate) as metrics.py:55-63 defines them."""
        false_pos_rate = self.FP / (self.FP + self.TN)
        false_neg_rate = self.FN / (self.FN + self.TP)
        return false_pos_rate, false_neg_rate

    def compute_f1(self):
        denom = (self.precision + self.recall).clamp(_CLAMP)
        return 2 * self.precision * self.recall / denom


# ------------------------------------------------------------------------------------------------
# functional helpers (metrics.py:62-145)
# ------------------------------------------------------------------------------------------------
def true_pos(y_true: torch.Tensor, y_pred: torch.Tensor, dim=0):
    return torch.sum(y_true * torch.round(y_pred), dim=dim)


def false_pos(y_true, y_pred, dim=0):
    return torch.sum((1. - y_true) * torch.round(y_pred), dim=dim)


def false_neg(y_true: torch.Tensor, y_pred: torch.Tensor, dim=0):
    return torch.sum(y_true * (1. - torch.round(y_pred)), dim=dim)


def precision(y_true: torch.Tensor, y_pred: torch.Tensor, dim: int):
    TP = true_pos(y_true, y_pred, dim)
    FP = false_pos(y_true, y_pred, dim)
    return TP / torch.clamp(TP + FP, _CLAMP)


def recall(y_true: torch.Tensor, y_pred: torch.Tensor, dim: int):
    TP = true_pos(y_true, y_pred, dim)
    FN = false_neg(y_true, y_pred, dim)
    return TP / torch.clamp(TP + FN, _CLAMP)


def f1_score(gts: torch.Tensor, preds: torch.Tensor, multi_threashold_mode=False, dim=(-1, -2)):
    gts = gts.float()
    preds = preds.float()
    if multi_threashold_mode:
        gts = gts[:, None, ...].expand_as(preds)
    with torch.no_grad():
        recall_val = recall(gts, preds, dim)
        precision_val = precision(gts, preds, dim)
        denom = torch.clamp(recall_val + precision_val, _CLAMP)
        return 2. * recall_val * precision_val / denom


def true_positives_from_prob(y_prob: np.ndarray, y_true: np.ndarray, threshold: float = 0.5):
    return np.sum(np.logical_and(y_prob > threshold, y_true))


def false_positives_from_prob(y_prob: np.ndarray, y_true: np.ndarray, threshold: float = 0.5):
    return np.sum(np.logical_and(y_prob > threshold, np.logical_not(y_true)))


def false_negatives_from_prob(y_prob: np.ndarray, y_true: np.ndarray, threshold: float = 0.5):
    return np.sum(np.logical_and(np.logical_not(y_prob > threshold), y_true))


def precsision_from_prob(y_prob: np.ndarray, y_true: np.ndarray, threshold: float = 0.5):
    tp = true_positives_from_prob(y_prob, y_true, threshold)
    fp = false_positives_from_prob(y_prob, y_true, threshold)
    return tp / (tp + fp)


def recall_from_prob(y_prob: np.ndarray, y_true: np.ndarray, threshold: float = 0.5):
    tp = true_positives_from_prob(y_prob, y_true, threshold)
    fn = false_negatives_from_prob(y_prob, y_true, threshold)
    return tp / (tp + fn)


def f1_score_from_prob(y_prob: np.ndarray, y_true: np.ndarray, threshold: float = 0.5):
    p = precsision_from_prob(y_prob, y_true, threshold=threshold)
    r = recall_from_prob(y_prob, y_true, threshold=threshold)
    return 2 * (p * r) / (p + r)


def root_mean_square_error(y_pred: np.ndarray, y_true: np.ndarray):
    return np.sqrt(np.sum(np.square(y_pred - y_true)) / np.size(y_true))
