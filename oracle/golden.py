"""ORACLE — TEST INFRASTRUCTURE ONLY.  Loading of the golden fixtures in tests/golden/*.npz.

The fixtures were produced by tests/golden/make_golden.py from the reference implementation itself;
this module only reads them (numpy.load with allow_pickle=False) and rebuilds configs.
"""
from __future__ import annotations

import json
import os

import numpy as np

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'tests', 'golden')
NAMES = ('siamese_t8-16', 'siamese_t8-16-32', 'unet_t8-16', 'dualstream_t8-16', 'dtsiamese_t8-16',
         'whatevernet_t8-16', 'siamese_t8-16-32_odd', 'dualstream_t8-16_odd', 'whatevernet2_t8-16',
         'siamese_t32-64', 'dtsiamese_t32-64', 'dualstream_t32-64', 'siamese_t12-20', 'dualstream_t6-12')


class Fixture:
    def __init__(self, name):
        self.name = name
        z = np.load(os.path.join(GOLDEN_DIR, f'{name}.npz'), allow_pickle=False)
        self.z = {k: z[k] for k in z.files}
        self.meta = json.loads(str(self.z['meta']))
        self.cfg = self.meta['cfg']
        self.model_type = self.cfg['TYPE']

    def prefixed(self, prefix):
        n = len(prefix)
        return {k[n:]: v for k, v in self.z.items() if k.startswith(prefix)}

    @property
    def params0(self):
        return self.prefixed('p0/')

    @property
    def grads(self):
        return self.prefixed('g/')

    @property
    def outputs(self):
        o = self.prefixed('out/')
        return [o[str(i)] for i in range(len(o))]

    @property
    def eval_outputs(self):
        o = self.prefixed('eval/')
        return [o[str(i)] for i in range(len(o))]

    def batch(self):
        import torch
        b = {k: torch.from_numpy(self.z[k]) for k in ('x_t1', 'x_t2', 'y_change', 'y_sem_t1', 'y_sem_t2')}
        b['is_labeled'] = torch.from_numpy(self.z['is_labeled'])
        return b

    def package_cfg(self):
        """A multimodal_siamese_cd_amd CfgNode for this fixture's model."""
        from multimodal_siamese_cd_amd.utils.experiment_manager import new_config
        c = new_config()
        c.MODEL.TYPE = self.model_type
        c.MODEL.IN_CHANNELS = self.cfg['IN_CHANNELS']
        c.MODEL.OUT_CHANNELS = self.cfg['OUT_CHANNELS']
        c.MODEL.TOPOLOGY = list(self.cfg['TOPOLOGY'])
        c.MODEL.LOSS_TYPE = 'PowerJaccardLoss'
        c.DATALOADER.S1_BANDS = list(self.cfg['S1_BANDS'])
        c.DATALOADER.S2_BANDS = list(self.cfg['S2_BANDS'])
        c.TRAINER.LR = self.meta['lr']
        c.CONSISTENCY_TRAINER.LOSS_FACTOR = self.meta['alpha']
        return c


def rel_err(a, b):
    """max|a - b| / max|b| (tensor-scale relative error)."""
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    den = max(np.abs(b).max(), 1e-30)
    return float(np.abs(a - b).max() / den)
