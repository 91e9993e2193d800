"""Data pipeline: MultimodalCDDataset over a tile cache + on-device augmentations.

CPU: AOI selection, labelled/unlabelled lists, multiplier, timestamp choice and label construction follow
utils/datasets.py:65-179; the augmentation draws consume a RandomState exactly as the reference's per-item chain
(oracle/augment_oracle.py) does, and pick the same importance crop.
GPU: device_collate's batched crop / flip / rot90 / colour shift / gamma equals the oracle chain item by item
(bit-exact; gamma within 1 fp32 ulp: device vs host libm pow).
"""
import os
import sys

import numpy as np
import pytest
import torch

from oracle import augment_oracle as A

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'tools'))
import make_tile_cache  # noqa: E402


def _cfg(root, aois, **aug):
    from multimodal_siamese_cd_amd.utils import experiment_manager as em
    cfg = em.load_cfg('baseline_siamese')
    cfg.PATHS.DATASET = str(root)
    cfg.DATASET.TRAINING_IDS = aois[:2]
    cfg.DATASET.VALIDATION_IDS = aois[2:]
    cfg.DATASET.UNLABELED_IDS = aois[2:]
    cfg.DATALOADER.TRAINING_MULTIPLIER = 2
    cfg.DATALOADER.S2_BANDS = [2, 1, 0]
    cfg.AUGMENTATION.CROP_SIZE = 64
    for k, v in aug.items():
        cfg.AUGMENTATION[k] = v
    return cfg


@pytest.fixture(scope='module')
def cache(tmp_path_factory):
    root = tmp_path_factory.mktemp('tiles')
    return root, make_tile_cache.make(str(root), aois=3, size=(100, 90), months=4)


def test_dataset_selection_and_items(cache):
    from multimodal_siamese_cd_amd.utils import datasets
    root, aois = cache
    cfg = _cfg(root, aois)
    cfg.DATALOADER.INCLUDE_UNLABELED = True
    ds = datasets.MultimodalCDDataset(cfg, 'training', dataset_mode='first_last')
    assert len(ds) == 6 and ds.labeled == [True, True, False] * 2
    assert ds.aoi_ids[:3] == aois[:2] + aois[2:]
    it = ds[0]  # aoi 0 has a masked second month: labelled timestamps skip it
    assert (it['year_t1'], it['month_t1'], it['year_t2'], it['month_t2']) == (2018, 1, 2018, 4)
    s1 = np.nan_to_num(np.clip(np.load(root / aois[0] / 's1' / f's1_{aois[0]}_2018_01.npy')[:, :, [0, 1]], 0, 1))
    assert np.array_equal(it['imgs'][:, :, :2], s1)
    b1 = np.load(root / aois[0] / 'buildings' / f'buildings_{aois[0]}_2018_01.npy') > 0
    b2 = np.load(root / aois[0] / 'buildings' / f'buildings_{aois[0]}_2018_04.npy') > 0
    assert np.array_equal(it['change'], (~b1 & b2).astype(np.float32))
    assert it['imgs'].shape[2] == 2 * 2 + 2 * 3 and it['is_labeled']
    un = ds[2]
    assert not un['is_labeled'] and not un['change'].any()
    assert len(datasets.MultimodalCDDataset(cfg, 'training', disable_multiplier=True, disable_unlabeled=True)) == 2


@pytest.mark.parametrize('aug', [dict(), dict(IMAGE_OVERSAMPLING_TYPE='none'),
                                 dict(COLOR_SHIFT=True, GAMMA_CORRECTION=True, RANDOM_ROTATE=False)])
def test_draws_consume_the_reference_random_stream(cache, aug):
    """After one item, the dataset's RandomState is where the reference chain leaves it, and the importance crop
    it would choose (window sums on the host here) is the chain's."""
    from multimodal_siamese_cd_amd.utils import augmentations, datasets
    root, aois = cache
    cfg = _cfg(root, aois, **aug)
    for seed in range(4):
        r1, r2 = np.random.RandomState(seed), np.random.RandomState(seed)
        ds = datasets.MultimodalCDDataset(cfg, 'training', rng=r1)
        it = ds[seed % len(ds)]
        n_ts = len([t for t in ds.metadata[it['aoi_id']] if t['s1'] and t['s2'] and t['buildings'] and not t['masked']])
        r2.randint(0, n_ts, size=2)  # the dataset's own timestamp draws (dataset_mode 'all')
        ref = A.chain(dict(cfg.AUGMENTATION), it['imgs'], it['buildings'], it['change'], r2)
        assert r1.get_state()[1].tolist() == r2.get_state()[1].tolist() and r1.get_state()[2] == r2.get_state()[2]
        d = it['aug']
        S = cfg.AUGMENTATION.CROP_SIZE
        if len(d.candidates) > 1:
            w = np.float32([it['change'][y:y + S, x:x + S].sum() for y, x in d.candidates]) + 5
            w = w / w.sum()
            cdf = w.astype(np.float64).cumsum()
            cdf /= cdf[-1]
            y, x = d.candidates[int(cdf.searchsorted(d.u, side='right'))]
        else:
            y, x = d.candidates[0]
        crop = it['change'][y:y + S, x:x + S]
        if d.flip_h:
            crop = np.flip(crop, 1)
        if d.flip_v:
            crop = np.flip(crop, 0)
        crop = np.rot90(crop, d.rot, axes=(0, 1))
        assert np.array_equal(np.ascontiguousarray(crop.transpose(2, 0, 1)), ref[2])


@pytest.mark.gpu
@pytest.mark.parametrize('aug', [dict(), dict(IMAGE_OVERSAMPLING_TYPE='none', RANDOM_ROTATE=False),
                                 dict(COLOR_SHIFT=True, GAMMA_CORRECTION=True)])
def test_device_augmentation_matches_reference_chain(cache, aug):
    from multimodal_siamese_cd_amd import hip
    from multimodal_siamese_cd_amd.utils import datasets
    hip.load_library()
    dev = torch.device('cuda:0')
    root, aois = cache
    cfg = _cfg(root, aois, **aug)
    cfg.DATALOADER.INCLUDE_BUILDING_LABELS = True
    ds = datasets.MultimodalCDDataset(cfg, 'training', rng=np.random.RandomState(11))
    items = [ds[i] for i in range(len(ds))]
    batch = datasets.device_collate(items, ds, dev)
    r2 = np.random.RandomState(11)
    for b, it in enumerate(items):
        n_ts = len([t for t in ds.metadata[it['aoi_id']] if t['s1'] and t['s2'] and t['buildings'] and not t['masked']])
        r2.randint(0, n_ts, size=2)
        imgs, bld, chg = A.chain(dict(cfg.AUGMENTATION), it['imgs'], it['buildings'], it['change'], r2)
        x_t1 = np.concatenate((imgs[0:2], imgs[4:7]))  # (s1_t1, s2_t1): datasets.py:157-158, 166-170
        x_t2 = np.concatenate((imgs[2:4], imgs[7:10]))
        for got, want in ((batch['x_t1'][b], x_t1), (batch['x_t2'][b], x_t2), (batch['y_change'][b], chg),
                          (batch['y_sem_t1'][b], bld[0:1]), (batch['y_sem_t2'][b], bld[1:2])):
            got = got.cpu().numpy()
            assert got.shape == want.shape
            if aug.get('GAMMA_CORRECTION'):
                assert np.all(np.abs(got - want) <= np.spacing(np.maximum(np.abs(want), 1e-30)))
            else:
                assert np.array_equal(got, want)
    assert batch['is_labeled'].tolist() == ds.labeled


@pytest.mark.gpu
def test_training_and_evaluation_on_the_tile_cache(cache, capsys):
    """train_supervised.run_training reads the tile cache (DATALOADER.SYNTHETIC: False), augments on the device and
    evaluates the validation/test AOIs as full tiles (evaluation.py:15-17)."""
    from multimodal_siamese_cd_amd import hip, train_supervised
    hip.load_library()
    root, aois = cache
    cfg = _cfg(root, aois)
    cfg.MODEL.TYPE, cfg.MODEL.TOPOLOGY = 'siameseunet', [64, 128]
    cfg.DATALOADER.SYNTHETIC = False
    cfg.DATALOADER.TRAINING_MULTIPLIER = 3
    cfg.DATASET.TEST_IDS = aois[2:]
    cfg.TRAINER.BATCH_SIZE, cfg.TRAINER.EPOCHS = 2, 1
    cfg.LOG_FREQ, cfg.DEBUG, cfg.SAVE_CHECKPOINTS = 100, False, []
    train_supervised.run_training(cfg, torch.device('cuda:0'))
    out = capsys.readouterr().out
    assert "'validation F1'" in out and "'test F1'" in out and 'epoch 1: mean loss' in out
