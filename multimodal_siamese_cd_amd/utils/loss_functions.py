"""Loss registry — drop-in for the reference's utils/loss_functions.py `get_criterion` (lines 6-33).

Only `PowerJaccardLoss` (loss_functions.py:141-150), the loss every reference config trains with
(configs/base.yaml:17, CONSISTENCY_TRAINER.LOSS_TYPE), is on the hot path; it runs as the fused
`scd_pjaccard_fwd/bwd` HIP kernels.  The other names the reference registers are recognised but not
built in this round (no config uses them) and raise NotImplementedError; unknown names raise like the
reference (`Exception('unknown loss ...')`).
"""
from __future__ import annotations

from .. import engine

_NOT_BUILT = ('BCEWithLogitsLoss', 'CrossEntropyLoss', 'SoftDiceLoss', 'SoftDiceSquaredSumLoss',
              'SoftDiceBalancedLoss', 'MeanSquareErrorLoss', 'IoULoss', 'DiceLikeLoss', 'L2')


def power_jaccard_loss(input, target):
    """1 - I / (sum(p^2 + t^2) - I + 1e-6), p = sigmoid(input), reduced over the whole batch."""
    return engine.power_jaccard(input, target)


def get_criterion(loss_type, negative_weight: float = 1, positive_weight: float = 1):
    if loss_type == 'PowerJaccardLoss':
        return power_jaccard_loss
    if loss_type in _NOT_BUILT:
        raise NotImplementedError(f'{loss_type} is not on the MI355X hot path (only PowerJaccardLoss is built)')
    raise Exception(f'unknown loss {loss_type}')
