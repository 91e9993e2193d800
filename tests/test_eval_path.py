"""Eval path: utils/evaluation.py:7-41 + utils/metrics.py:5-59 + the Up zero-pad path.

CPU: the metric oracle is pinned to tests/golden/metrics_mt.npz (made by running the reference's utils/metrics.py),
and the host-side accumulation of MultiThresholdMetric reproduces the reference's float32 totals bit-exactly from
exact integer counts.
GPU: scd_threshold_counts is bit-exact against the oracle (integer work); scd_window_copy is bit-exact against
F.pad; model_evaluation's F1 equals the oracle's eval-mode forward scored by the oracle metric, on tiles whose sizes
are not divisible by 2**levels (the Up pad path).  The odd-size model fixtures (siamese_t8-16-32_odd,
dualstream_t8-16_odd) run through tests/test_model_gpu.py's train/eval parity tests.
"""
import numpy as np
import pytest
import torch

from oracle import metrics_oracle as M
from oracle.golden import GOLDEN_DIR

FIX = f'{GOLDEN_DIR}/metrics_mt.npz'


def _fixture():
    z = np.load(FIX, allow_pickle=False)
    return {k: z[k] for k in z.files}


def test_metric_oracle_matches_reference_fixture():
    z = _fixture()
    for prefix, thr in (('', z['thresholds']), ('eval_', np.float32([0.5]))):
        tot = {k: np.zeros(len(thr), np.float32) for k in ('TP', 'TN', 'FP', 'FN')}
        for i in range(3):
            c = M.confusion(z[f'y_true/{i}'], z[f'y_pred/{i}'], thr)
            for k in tot:
                tot[k] = tot[k] + c[k].astype(np.float32)
        for k in tot:
            assert np.array_equal(tot[k], z[prefix + k]), (prefix, k)


def test_multithreshold_accumulation_is_bit_exact():
    """MultiThresholdMetric's float32 bookkeeping on exact counts == the reference's totals and derived metrics."""
    from multimodal_siamese_cd_amd.utils import metrics
    z = _fixture()
    m = metrics.MultiThresholdMetric(torch.from_numpy(z['thresholds']))
    for i in range(3):
        y, p = z[f'y_true/{i}'], z[f'y_pred/{i}']
        m._accumulate(torch.from_numpy(M.kernel_counts(y, p, z['thresholds'])), p.size)
    for k in ('TP', 'TN', 'FP', 'FN'):
        assert np.array_equal(getattr(m, k).numpy(), z[k]), k
    assert np.array_equal(m.precision.numpy(), z['precision'])
    assert np.array_equal(m.recall.numpy(), z['recall'])
    assert np.array_equal(m.compute_f1().numpy(), z['f1'])
    fpr, fnr = m.compute_basic_metrics()
    assert np.array_equal(fpr.numpy(), z['fpr'], equal_nan=True)
    assert np.array_equal(fnr.numpy(), z['fnr'], equal_nan=True)


def test_counts_layout_roundtrip():
    from multimodal_siamese_cd_amd.utils import metrics
    rng = np.random.default_rng(3)
    p = rng.random(1000, dtype=np.float32)
    y = (rng.random(1000) > 0.5).astype(np.float32)
    thr = np.float32([0.1, 0.5, 0.9])
    tp, tn, fp, fn = metrics.confusion_from_counts(torch.from_numpy(M.kernel_counts(y, p, thr)), p.size)
    c = M.confusion(y, p, thr)
    for a, k in zip((tp, tn, fp, fn), ('TP', 'TN', 'FP', 'FN')):
        assert np.array_equal(a.numpy(), c[k])


def test_pad_window_oracle_matches_fpad():
    import torch.nn.functional as F
    x = torch.randn(2, 3, 5, 7)  # NCHW, H=5, W=7
    for h, w in ((5, 7), (6, 7), (5, 9), (8, 10)):
        dy, dx = h - 5, w - 7
        ref = F.pad(x, (dx // 2, dx - dx // 2, dy // 2, dy - dy // 2)).permute(0, 2, 3, 1).numpy()
        got = M.pad_window(x.permute(0, 2, 3, 1).numpy(), h, w)
        assert np.array_equal(got, ref)


def test_product_metric_refuses_cpu_tensors():
    from multimodal_siamese_cd_amd.utils import metrics
    m = metrics.MultiThresholdMetric(torch.tensor([0.5]))
    with pytest.raises(RuntimeError):
        m.add_sample(torch.zeros(1, 1, 4, 4), torch.zeros(1, 1, 4, 4))


# ------------------------------------------------------------------------------------------------
# GPU
# ------------------------------------------------------------------------------------------------
@pytest.fixture(scope='module')
def dev():
    from multimodal_siamese_cd_amd import hip
    hip.load_library()
    d = torch.device('cuda:0')
    hip.ensure_device(torch.empty(1, device=d))
    return d


@pytest.mark.gpu
@pytest.mark.parametrize('n', [1, 3, 4, 1027, 65536 + 5, 3 * 1024 * 1024 + 2])
@pytest.mark.parametrize('n_thr', [1, 5, 16])
def test_threshold_counts_bit_exact(dev, n, n_thr):
    from multimodal_siamese_cd_amd import hip
    rng = np.random.default_rng(n + 17 * n_thr)
    p = rng.random(n, dtype=np.float32)
    thr = np.sort(rng.random(n_thr, dtype=np.float32))
    thr[0] = 0.5
    k = min(n, 3 * n_thr)
    p[:k] = np.concatenate([thr, np.nextafter(thr, 2), np.nextafter(thr, -1)])[:k]  # exact ties
    if n > 8:
        p[5] = np.nan
    y = (rng.random(n) > 0.7).astype(np.float32)
    if n > 9:
        y[9] = np.nan
    pt, yt, tt = (torch.from_numpy(a).to(dev) for a in (p, y, thr))
    counts = torch.empty(1 + 2 * n_thr, dtype=torch.int64, device=dev)
    ws = torch.empty(hip.threshold_counts_workspace_bytes(n, n_thr), dtype=torch.uint8, device=dev)
    hip.threshold_counts(pt, yt, tt, False, counts, ws)
    assert np.array_equal(counts.cpu().numpy(), M.kernel_counts(y, p, thr))


@pytest.mark.gpu
def test_threshold_counts_from_logits(dev):
    """Fused sigmoid: equal to counting sigmoid(logit) except where the probability sits within 2 ulp of a
    threshold (the device expf and the CPU sigmoid may round differently there).  The input includes 129 logits
    straddling each threshold, so that band is populated and the bound is exercised, not vacuous."""
    from multimodal_siamese_cd_amd import hip
    rng = np.random.default_rng(5)
    n = 1 << 20
    thr = np.float32([0.5, 0.25, 0.75, 0.9])
    # logits placed on the thresholds: logit(t) and its 64 fp32 neighbours either side
    edge = []
    for t in thr.astype(np.float64):
        x0 = np.float32(np.log(t / (1 - t)))
        up, dn = [x0], [x0]
        for _ in range(64):
            up.append(np.nextafter(up[-1], np.float32(np.inf)))
            dn.append(np.nextafter(dn[-1], np.float32(-np.inf)))
        edge += up + dn[1:]
    edge = np.array(edge, dtype=np.float32)
    x = np.concatenate([(rng.standard_normal(n - edge.size) * 4).astype(np.float32), edge])
    y = (rng.random(n) > 0.8).astype(np.float32)
    p = torch.sigmoid(torch.from_numpy(x)).numpy()
    counts = torch.empty(1 + 2 * thr.size, dtype=torch.int64, device=dev)
    ws = torch.empty(hip.threshold_counts_workspace_bytes(n, thr.size), dtype=torch.uint8, device=dev)
    hip.threshold_counts(torch.from_numpy(x).to(dev), torch.from_numpy(y).to(dev), torch.from_numpy(thr).to(dev), True,
                         counts, ws)
    got = counts.cpu().numpy()
    ref = M.kernel_counts(y, p, thr)
    near = [int(np.sum(np.abs(p - t) <= 2 * np.spacing(t))) for t in thr]
    assert got[0] == ref[0]
    for k in range(thr.size):
        assert abs(got[1 + 2 * k] - ref[1 + 2 * k]) <= near[k]
        assert abs(got[2 + 2 * k] - ref[2 + 2 * k]) <= near[k]


@pytest.mark.gpu
def test_multithreshold_metric_matches_reference_fixture(dev):
    from multimodal_siamese_cd_amd.utils import metrics
    z = _fixture()
    m = metrics.MultiThresholdMetric(torch.from_numpy(z['thresholds']))
    m5 = metrics.MultiThresholdMetric(torch.linspace(0.5, 1, 1))
    for i in range(3):
        y = torch.from_numpy(z[f'y_true/{i}']).to(dev)
        p = torch.from_numpy(z[f'y_pred/{i}']).to(dev)
        m.add_sample(y, p)
        m5.add_sample(y, p)
    for k in ('TP', 'TN', 'FP', 'FN'):
        assert np.array_equal(getattr(m, k).cpu().numpy(), z[k]), k
        assert np.array_equal(getattr(m5, k).cpu().numpy(), z['eval_' + k]), k
    np.testing.assert_allclose(m.compute_f1().cpu().numpy(), z['f1'], rtol=1e-6, atol=0)
    np.testing.assert_allclose(m.precision.cpu().numpy(), z['precision'], rtol=1e-6, atol=0)
    np.testing.assert_allclose(m.recall.cpu().numpy(), z['recall'], rtol=1e-6, atol=0)
    np.testing.assert_allclose(m5.compute_f1().cpu().numpy(), z['eval_f1'], rtol=1e-6, atol=0)


@pytest.mark.gpu
def test_metric_more_than_16_thresholds(dev):
    from multimodal_siamese_cd_amd.utils import metrics
    rng = np.random.default_rng(9)
    p = rng.random((2, 1, 33, 17), dtype=np.float32)
    y = (rng.random((2, 1, 33, 17)) > 0.5).astype(np.float32)
    thr = torch.linspace(0, 1, 37)
    m = metrics.MultiThresholdMetric(thr)
    m.add_sample(torch.from_numpy(y).to(dev), torch.from_numpy(p).to(dev))
    c = M.confusion(y, p, thr.numpy())
    for k in ('TP', 'TN', 'FP', 'FN'):
        assert np.array_equal(getattr(m, k).cpu().numpy(), c[k].astype(np.float32)), k


@pytest.mark.gpu
@pytest.mark.parametrize('shape,oy,ox', [((2, 9, 11, 8), -1, 0), ((1, 18, 22, 16), 0, -1), ((3, 5, 7, 4), -2, -3),
                                         ((2, 36, 44, 8), 1, 1), ((1, 4, 4, 12), 0, 0)])
def test_window_copy_matches_fpad(dev, shape, oy, ox):
    """Forward (negative offsets: pad) into a channel slice of a wider buffer, and backward (positive: crop)."""
    from multimodal_siamese_cd_amd import hip
    n, h, w, c = shape
    rng = np.random.default_rng(h * w)
    if oy <= 0 and ox <= 0:  # pad a (h + 2|oy| - 1 ...) map: the up map is smaller than the destination
        hu, wu = h - 2 * (-oy) - (1 if oy else 0), w - 2 * (-ox) - (1 if ox else 0)
        hu, wu = max(hu, 1), max(wu, 1)
        up = rng.standard_normal((n, hu, wu, c)).astype(np.float32)
        dst = torch.full((n, h, w, c + 8), 7.0, device=dev)
        hip.window_copy(hip.nhwc(torch.from_numpy(up).to(dev)), hip.nhwc(dst, 8, c), oy, ox)
        ref = np.zeros((n, h, w, c), np.float32)
        ref[:, -oy:-oy + hu, -ox:-ox + wu] = up
        got = dst.cpu().numpy()
        assert np.array_equal(got[..., 8:], ref)
        assert np.all(got[..., :8] == 7.0)
    else:
        src = rng.standard_normal((n, h + 2 * oy + 1, w + 2 * ox + 1, c + 4)).astype(np.float32)
        st = torch.from_numpy(src).to(dev)
        dst = torch.empty((n, h, w, c), device=dev)
        hip.window_copy(hip.nhwc(st, 4, c), hip.nhwc(dst), oy, ox)
        assert np.array_equal(dst.cpu().numpy(), src[:, oy:oy + h, ox:ox + w, 4:])


@pytest.mark.gpu
def test_model_evaluation_matches_oracle_on_odd_tiles(dev):
    """evaluation.model_evaluation (utils/evaluation.py:7-41) on AOI-like tiles whose sizes are not divisible by
    2**levels: F1 / precision / recall equal the oracle's eval-mode forward scored by the oracle metric."""
    from multimodal_siamese_cd_amd.utils import evaluation, networks
    from oracle import siamese_oracle as O
    from oracle.golden import Fixture
    fx = Fixture('siamese_t8-16-32_odd')
    cfg = fx.package_cfg()
    net = networks.create_network(cfg)
    P = {k: torch.from_numpy(v.copy()) for k, v in fx.params0.items()}
    B = O.fresh_buffers(O.param_shapes(fx.model_type, fx.cfg))
    rng = np.random.default_rng(11)
    for k, b in B.items():  # non-trivial running statistics
        if k.endswith('running_mean'):
            b.copy_(torch.from_numpy(rng.standard_normal(b.shape).astype(np.float32) * 0.1))
        elif k.endswith('running_var'):
            b.copy_(torch.from_numpy(rng.random(b.shape, dtype=np.float32) + 0.5))
    with torch.no_grad():
        for k, p in net.module.named_parameters():
            p.copy_(P[k])
        sd = net.module.state_dict()
        for k, b in B.items():
            sd[k].copy_(b)
    items = []
    for i, (h, w) in enumerate([(37, 45), (50, 29), (64, 64)]):
        g = torch.Generator().manual_seed(100 + i)
        c = fx.cfg['IN_CHANNELS']
        items.append({'x_t1': torch.rand(c, h, w, generator=g), 'x_t2': torch.rand(c, h, w, generator=g),
                      'y_change': (torch.rand(1, h, w, generator=g) > 0.8).float()})
    thr = np.float32([0.3, 0.5, 0.7])
    res = evaluation.model_evaluation(net, cfg, dev, 'validation', 1.0, 10, dataset=items, log=lambda d: None,
                                      thresholds=thr)
    tot = {k: np.zeros(3, np.float32) for k in ('TP', 'TN', 'FP', 'FN')}
    margin = 0
    for it in items:
        with torch.no_grad():
            lg = O.forward(fx.model_type, P, B, it['x_t1'][None], it['x_t2'][None], fx.cfg, training=False)
        p = torch.sigmoid(lg).numpy()
        margin += sum(int(np.sum(np.abs(p - t) < 1e-5)) for t in thr)  # pixels a 1e-5 logit wobble could flip
        c = M.confusion(it['y_change'][None].numpy(), p, thr)
        for k in tot:
            tot[k] = tot[k] + c[k].astype(np.float32)
    prec = tot['TP'] / np.maximum(tot['TP'] + tot['FP'], np.float32(10e-05))
    rec = tot['TP'] / np.maximum(tot['TP'] + tot['FN'], np.float32(10e-05))
    f1 = 2 * prec * rec / np.maximum(prec + rec, np.float32(10e-05))
    j = int(np.argmax(f1))
    # each flipped pixel moves a ratio by at most ~2 / its denominator
    den = float(min(tot['TP'][j] + tot['FP'][j], tot['TP'][j] + tot['FN'][j]))
    tol = 2.0 * margin / max(den, 1.0) + 1e-6
    print('eval', res, 'oracle F1', f1, 'near-threshold pixels', margin)
    assert abs(res['validation F1'] - float(f1[j])) <= tol, (res, f1, margin)
    assert abs(res['validation precision'] - float(prec[j])) <= tol
    assert abs(res['validation recall'] - float(rec[j])) <= tol


@pytest.mark.gpu
def test_training_loop_runs_evaluation(dev, capsys):
    """train_supervised.run_training calls model_evaluation at LOG_FREQ and at the epoch end
    (train_supervised.py:84-113) on full tiles of an odd size."""
    from multimodal_siamese_cd_amd import train_supervised
    from multimodal_siamese_cd_amd.utils import datasets, experiment_manager as em
    cfg = em.load_cfg('debug')
    cfg.DEBUG = False
    cfg.TRAINER.EPOCHS = 1
    cfg.TRAINER.STEPS_PER_EPOCH = 2
    cfg.LOG_FREQ = 1
    cfg.EVAL_SAMPLES = 1
    cfg.SAVE_CHECKPOINTS = []
    orig = datasets.SyntheticCDDataset.__init__

    def odd_tiles(self, *a, **kw):
        kw['size'] = (70, 52)
        orig(self, *a, **kw)
    datasets.SyntheticCDDataset.__init__ = odd_tiles
    try:
        train_supervised.run_training(cfg, dev)
    finally:
        datasets.SyntheticCDDataset.__init__ = orig
    out = capsys.readouterr().out
    for rt in ('training', 'validation', 'test'):
        assert f"'{rt} F1'" in out, out
    assert out.count("'validation F1'") == 3  # step 1, step 2, epoch end
