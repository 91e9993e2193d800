"""Per-step loss recipes of the reference trainers, on the HIP path.

  supervised  train_supervised.py:63-79            loss = criterion(logits, y_change)
  dual task   train_supervised_dualtask.py:64-90   (L_change + (L_sem_t1 + L_sem_t2) / 2) / 2
  MMCR        train_semisupervised.py:66-121       alpha * mean(L_fusion, L_s1, L_s2) on labelled samples
                                                   + (1 - alpha) * PJ(logits_s1, sigmoid(logits_s2)) on unlabelled
                                                   (the soft target is NOT detached, as in the reference)
"""
from __future__ import annotations

import torch

from . import engine
from .utils import loss_functions


def _fusable(*criteria) -> bool:
    return all(c is loss_functions.power_jaccard_loss for c in criteria)


def supervised_loss(criterion, logits, batch):
    return criterion(logits, batch['y_change'])


def dualtask_loss(change_criterion, sem_criterion, outputs, batch):
    logits_change, logits_sem_t1, logits_sem_t2 = outputs
    if _fusable(change_criterion, sem_criterion):  # one fused pass: 0.5 L_change + 0.25 L_sem_t1 + 0.25 L_sem_t2
        lab = torch.ones(logits_change.shape[0], dtype=torch.uint8, device=logits_change.device)
        spec = [(0, 1, 0.5, 0, 0), (2, 3, 0.25, 0, 0), (4, 5, 0.25, 0, 0)]
        return engine.multi_jaccard(spec, lab, logits_change, batch['y_change'], logits_sem_t1, batch['y_sem_t1'],
                                    logits_sem_t2, batch['y_sem_t2'])
    change_loss = change_criterion(logits_change, batch['y_change'])
    sem_loss = (sem_criterion(logits_sem_t1, batch['y_sem_t1']) + sem_criterion(logits_sem_t2, batch['y_sem_t2'])) / 2
    return (change_loss + sem_loss) / 2


def mmcr_loss(sup_criterion, cons_criterion, outputs, batch, alpha: float, cons_loss_type: str = 'PowerJaccardLoss'):
    logits_fusion, logits_s1, logits_s2 = outputs
    is_labeled = batch['is_labeled'].to(logits_fusion.device)
    y = batch['y_change']
    if cons_loss_type != 'L2' and _fusable(sup_criterion, cons_criterion):
        # one fused pass, subsets selected on the device: alpha/3 * (L_f + L_s1 + L_s2)[labelled]
        # + (1 - alpha) * PJ(logits_s1, sigmoid(logits_s2))[unlabelled]
        a = float(alpha)
        spec = [(0, 3, a / 3, 1, 0), (1, 3, a / 3, 1, 0), (2, 3, a / 3, 1, 0), (1, 2, 1 - a, 2, 1)]
        return engine.multi_jaccard(spec, is_labeled, logits_fusion, logits_s1, logits_s2, y)
    loss = None
    if bool(is_labeled.any()):
        sup = (sup_criterion(logits_fusion[is_labeled], y[is_labeled])
               + sup_criterion(logits_s1[is_labeled], y[is_labeled])
               + sup_criterion(logits_s2[is_labeled], y[is_labeled])) / 3
        loss = alpha * sup
    if not bool(is_labeled.all()):
        nl = torch.logical_not(is_labeled)
        if cons_loss_type == 'L2':
            raise NotImplementedError('L2 consistency loss is not on the MI355X hot path')
        cons = (1 - alpha) * cons_criterion(logits_s1[nl], torch.sigmoid(logits_s2[nl]))
        loss = cons if loss is None else loss + cons
    return loss


def step_loss(cfg, outputs, batch, net=None):
    """Dispatch on the model family the way the reference's three trainers do.  `net`: the (wrapped) model the
    outputs come from; a model wrapped with exact_dataparallel=True forms ONE loss over the batch of all ranks
    (parallel.loss_scope), any other loss stays local."""
    from . import parallel
    with parallel.loss_scope(net):
        return _step_loss(cfg, outputs, batch)


def _step_loss(cfg, outputs, batch):
    t = cfg.MODEL.TYPE
    crit = loss_functions.get_criterion(cfg.MODEL.LOSS_TYPE)
    if t == 'dtsiameseunet':
        return dualtask_loss(crit, crit, outputs, batch)
    if t in ('whatevernet', 'whatevernet2') and isinstance(outputs, (tuple, list)):
        cons_type = cfg.CONSISTENCY_TRAINER.get('LOSS_TYPE', 'PowerJaccardLoss')
        cons = loss_functions.get_criterion(cons_type) if cons_type != 'L2' else None
        return mmcr_loss(crit, cons, outputs, batch, cfg.CONSISTENCY_TRAINER.LOSS_FACTOR, cons_type)
    return supervised_loss(crit, outputs, batch)
