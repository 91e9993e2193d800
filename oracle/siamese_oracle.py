"""ORACLE — TEST INFRASTRUCTURE ONLY.  Never imported by the product package.

A from-scratch, functional CPU restatement (torch fp32 on CPU) of the reference's hot path, written
from the reference's source (SebastianHafner/multimodal_siamese_cd):

  DoubleConv      utils/networks.py:386-402   conv3x3(pad 1, bias) -> BN(train/eval) -> ReLU, twice
  InConv          utils/networks.py:405-412
  Down            utils/networks.py:415-426   MaxPool2d(2) -> DoubleConv
  Encoder         utils/networks.py:313-343   returns [x, down1, ..., downL] reversed
  Up              utils/networks.py:429-451   ConvT(2, s2) -> F.pad to skip -> cat([skip, up]) -> DoubleConv
  Decoder         utils/networks.py:346-382   pops the deepest feature, then up{L}..up1
  OutConv         utils/networks.py:454-461   conv1x1
  SiameseUNet     utils/networks.py:123-154   shared inc/encoder on t1 then t2, diff t2 - t1, decoder, head
  UNet            utils/networks.py:59-79     early fusion cat(t1, t2)
  DualStreamUNet  utils/networks.py:82-120    per-modality early fusion, cat of decoders -> head
  DualTaskSiameseUNet utils/networks.py:157-197
  WhateverNet     utils/networks.py:200-263   per-modality Siamese streams + fusion head
  WhateverNet2    utils/networks.py:266-310   per-modality early-fusion streams, per-stream heads + fusion head
  power_jaccard_loss  utils/loss_functions.py:141-150

Parameters are a flat dict keyed by the reference's state_dict names (without the `module.` prefix);
BatchNorm buffers live in a second dict and are updated in place like nn.BatchNorm2d's.

Parity pinning: tests/golden/make_golden.py runs the *reference itself* (imported from /root/reference in
the build container) and commits the outputs as .npz fixtures; tests/test_oracle_golden.py checks this
restatement against them.  The GPU tests compare the HIP path against this oracle and the fixtures.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

BN_EPS = 1e-5
BN_MOMENTUM = 0.1


# --------------------------------------------------------------------------------------------------
# topology helpers (utils/networks.py:313-382)
# --------------------------------------------------------------------------------------------------
def encoder_channels(topology):
    """Output channels of inc, down1..downL (networks.py:323-330)."""
    n = len(topology)
    return [topology[0]] + [topology[i + 1] if i != n - 1 else topology[i] for i in range(n)]


def decoder_layers(topology):
    """[(name, in_ch, out_ch)] in module order up{L}..up1 (networks.py:354-370)."""
    n = len(topology)
    up_topo = encoder_channels(topology)
    out = []
    for idx in reversed(range(n)):
        x2 = idx - 1 if idx != 0 else idx
        out.append((f'up{idx + 1}', up_topo[idx] * 2, up_topo[x2]))
    return out


# --------------------------------------------------------------------------------------------------
# blocks
# --------------------------------------------------------------------------------------------------
RECORD = None  # set to a list to capture (bn key, pre-activation) pairs (used to find ReLU-kink pixels)
# Branch matching (test infrastructure, tests/_parity.py BranchMatch): BRANCH(bn key, pre-activation) -> (mask, a)
# gives the ReLU decisions (bool, the pre-activation's shape) and the fp32 activation an implementation under test
# took at that BatchNorm output.  _relu then follows those decisions (y where mask, else 0; the gradient through
# the mask) and the MaxPool2d after it takes that activation's argmax (first maximum of each 2x2 window, as
# torch's CPU max_pool2d), so the oracle computes the gradient of the same piecewise-linear branch.
BRANCH = None
_LAST_A = None


def _relu(y, key):
    global _LAST_A
    if BRANCH is None:
        return F.relu(y)
    m, _LAST_A = BRANCH(key, y)
    return torch.where(m, y, torch.zeros_like(y))


def _windows(t):
    """(n, c, h, w) -> (n, c, h // 2, w // 2, 4): the 2x2 windows of MaxPool2d(2) (floor), (dy, dx) row-major."""
    n, c, h, w = t.shape
    h2, w2 = h // 2, w // 2
    return t[:, :, :2 * h2, :2 * w2].reshape(n, c, h2, 2, w2, 2).permute(0, 1, 2, 4, 3, 5).reshape(n, c, h2, w2, 4)


def _maxpool2(x):
    """MaxPool2d(2) (networks.py:421); under BRANCH the window argmaxes of the matched activation."""
    if BRANCH is None:
        return F.max_pool2d(x, 2)
    idx = _windows(_LAST_A).argmax(-1, keepdim=True)
    return _windows(x).gather(-1, idx).squeeze(-1)


def _bn(x, P, B, key, training):
    rm, rv = B[key + '.running_mean'], B[key + '.running_var']
    y = F.batch_norm(x, rm, rv, P[key + '.weight'], P[key + '.bias'], training, BN_MOMENTUM, BN_EPS)
    if RECORD is not None:
        RECORD.append((key, y.detach()))
    if training:
        B[key + '.num_batches_tracked'] += 1
    return y


def double_conv(x, P, B, pre, training):
    """utils/networks.py:386-402."""
    x = F.conv2d(x, P[pre + 'conv.0.weight'], P[pre + 'conv.0.bias'], padding=1)
    x = _relu(_bn(x, P, B, pre + 'conv.1', training), pre + 'conv.1')
    x = F.conv2d(x, P[pre + 'conv.3.weight'], P[pre + 'conv.3.bias'], padding=1)
    x = _relu(_bn(x, P, B, pre + 'conv.4', training), pre + 'conv.4')
    return x


def encoder(x, P, B, inc, enc, topology, training):
    """InConv (405-412) + Encoder (313-343); returns the reversed feature list like Encoder.forward."""
    feats = [double_conv(x, P, B, inc + 'conv.', training)]
    for i in range(len(topology)):
        pooled = _maxpool2(feats[-1])  # the activation of the last _relu
        feats.append(double_conv(pooled, P, B, f'{enc}down_seq.down{i + 1}.mpconv.1.', training))
    return feats[::-1]


def up(x1, x2, P, B, pre, training):
    """utils/networks.py:436-451."""
    x1 = F.conv_transpose2d(x1, P[pre + 'up.weight'], P[pre + 'up.bias'], stride=2)
    dy = x2.size(2) - x1.size(2)
    dx = x2.size(3) - x1.size(3)
    x1 = F.pad(x1, (dx // 2, dx - dx // 2, dy // 2, dy - dy // 2))
    return double_conv(torch.cat([x2, x1], dim=1), P, B, pre + 'conv.', training)


def decoder(features, P, B, dec, topology, training):
    """utils/networks.py:375-382 (works on a copy: the reference pops its argument in place)."""
    features = list(features)
    x1 = features.pop(0)
    for k, (name, _, _) in enumerate(decoder_layers(topology)):
        x1 = up(x1, features[k], P, B, f'{dec}up_seq.{name}.', training)
    return x1


def out_conv(x, P, pre):
    return F.conv2d(x, P[pre + 'conv.weight'], P[pre + 'conv.bias'])


def diff(f1, f2):
    return [torch.sub(b, a) for a, b in zip(f1, f2)]


# --------------------------------------------------------------------------------------------------
# models (forward only; gradients via torch autograd on CPU)
# --------------------------------------------------------------------------------------------------
def forward(model_type, P, B, x_t1, x_t2, cfg, training=True):
    topo = list(cfg['TOPOLOGY'])
    n1 = len(cfg['S1_BANDS'])
    if model_type == 'siameseunet':
        f1 = encoder(x_t1, P, B, 'inc.', 'encoder.', topo, training)
        f2 = encoder(x_t2, P, B, 'inc.', 'encoder.', topo, training)
        return out_conv(decoder(diff(f1, f2), P, B, 'decoder.', topo, training), P, 'outc.')
    if model_type == 'unet':
        x = torch.cat((x_t1, x_t2), dim=1)
        f = encoder(x, P, B, 'inc.', 'encoder.', topo, training)
        return out_conv(decoder(f, P, B, 'decoder.', topo, training), P, 'outc.')
    if model_type == 'dualstreamunet':
        outs = []
        for s, (a, b) in ((1, (x_t1[:, :n1], x_t2[:, :n1])), (2, (x_t1[:, n1:], x_t2[:, n1:]))):
            x = torch.cat((a, b), dim=1)
            f = encoder(x, P, B, f'inc_stream{s}.', f'encoder_stream{s}.', topo, training)
            outs.append(decoder(f, P, B, f'decoder_stream{s}.', topo, training))
        return out_conv(torch.cat(outs, dim=1), P, 'outc.')
    if model_type == 'dtsiameseunet':
        f1 = encoder(x_t1, P, B, 'inc.', 'encoder.', topo, training)
        f2 = encoder(x_t2, P, B, 'inc.', 'encoder.', topo, training)
        out_change = out_conv(decoder(diff(f1, f2), P, B, 'decoder_change.', topo, training), P, 'outc_change.')
        out_sem_t2 = out_conv(decoder(f2, P, B, 'decoder_sem.', topo, training), P, 'outc_sem.')
        out_sem_t1 = out_conv(decoder(f1, P, B, 'decoder_sem.', topo, training), P, 'outc_sem.')
        return out_change, out_sem_t1, out_sem_t2
    if model_type == 'whatevernet':
        decs, outs = [], []
        for s, (a, b) in ((1, (x_t1[:, :n1], x_t2[:, :n1])), (2, (x_t1[:, n1:], x_t2[:, n1:]))):
            f1 = encoder(a, P, B, f'inc_stream{s}.', f'encoder_stream{s}.', topo, training)
            f2 = encoder(b, P, B, f'inc_stream{s}.', f'encoder_stream{s}.', topo, training)
            d = decoder(diff(f1, f2), P, B, f'decoder_stream{s}.', topo, training)
            decs.append(d)
            outs.append(out_conv(d, P, f'outc_stream{s}.'))
        fusion = out_conv(torch.cat(decs, dim=1), P, 'outc_fusion.')
        return (fusion, outs[0], outs[1]) if training else fusion
    if model_type == 'whatevernet2':  # networks.py:288-310
        decs, outs = [], []
        for s, (a, b) in ((1, (x_t1[:, :n1], x_t2[:, :n1])), (2, (x_t1[:, n1:], x_t2[:, n1:]))):
            f = encoder(torch.cat((a, b), dim=1), P, B, f'inc_stream{s}.', f'encoder_stream{s}.', topo, training)
            d = decoder(f, P, B, f'decoder_stream{s}.', topo, training)
            decs.append(d)
            outs.append(out_conv(d, P, f'outc_stream{s}.'))
        fusion = out_conv(torch.cat(decs, dim=1), P, 'outc_fusion.')
        return (fusion, outs[0], outs[1]) if training else fusion
    raise ValueError(f'oracle: unsupported model {model_type}')


# --------------------------------------------------------------------------------------------------
# loss + trainer recipes
# --------------------------------------------------------------------------------------------------
def power_jaccard_loss(inp, target):
    """utils/loss_functions.py:141-150."""
    p = torch.sigmoid(inp).flatten()
    t = target.flatten()
    inter = (p * t).sum()
    denom = (p ** 2 + t ** 2).sum() - (p * t).sum() + 1e-6
    return 1 - inter / denom


def step_loss(model_type, outputs, batch, alpha=0.5):
    """The loss each reference trainer builds from the model outputs.

    supervised    train_supervised.py:71-75
    dual task     train_supervised_dualtask.py:71-85  (change + mean of the two semantic losses) / 2
    MMCR          train_semisupervised.py:74-119      alpha * mean(sup losses) on labelled samples
                                                      + (1 - alpha) * PJ(logits_s1, sigmoid(logits_s2)) on the rest
    """
    y = batch['y_change']
    if model_type in ('siameseunet', 'unet', 'dualstreamunet'):
        return power_jaccard_loss(outputs, y)
    if model_type == 'dtsiameseunet':
        out_change, out_sem_t1, out_sem_t2 = outputs
        lc = power_jaccard_loss(out_change, y)
        ls = (power_jaccard_loss(out_sem_t1, batch['y_sem_t1']) + power_jaccard_loss(out_sem_t2, batch['y_sem_t2'])) / 2
        return (lc + ls) / 2
    if model_type in ('whatevernet', 'whatevernet2'):
        fusion, s1, s2 = outputs
        lab = batch['is_labeled']
        loss = None
        if lab.any():
            sup = (power_jaccard_loss(fusion[lab], y[lab]) + power_jaccard_loss(s1[lab], y[lab])
                   + power_jaccard_loss(s2[lab], y[lab])) / 3
            loss = alpha * sup
        if not lab.all():
            nl = ~lab
            cons = (1 - alpha) * power_jaccard_loss(s1[nl], torch.sigmoid(s2[nl]))
            loss = cons if loss is None else loss + cons
        return loss
    raise ValueError(model_type)


# --------------------------------------------------------------------------------------------------
# parameter / buffer construction with the reference's names and shapes
# --------------------------------------------------------------------------------------------------
def _dc_shapes(pre, cin, cout):
    return {
        pre + 'conv.0.weight': (cout, cin, 3, 3), pre + 'conv.0.bias': (cout,),
        pre + 'conv.1.weight': (cout,), pre + 'conv.1.bias': (cout,),
        pre + 'conv.3.weight': (cout, cout, 3, 3), pre + 'conv.3.bias': (cout,),
        pre + 'conv.4.weight': (cout,), pre + 'conv.4.bias': (cout,),
    }


def _stream_shapes(inc, enc, dec, cin, topo):
    s = _dc_shapes(inc + 'conv.', cin, topo[0])
    ch = encoder_channels(topo)
    for i in range(len(topo)):
        s.update(_dc_shapes(f'{enc}down_seq.down{i + 1}.mpconv.1.', ch[i], ch[i + 1]))
    for name, cin_, cout in decoder_layers(topo):
        half = cin_ // 2
        s[f'{dec}up_seq.{name}.up.weight'] = (half, half, 2, 2)
        s[f'{dec}up_seq.{name}.up.bias'] = (half,)
        s.update(_dc_shapes(f'{dec}up_seq.{name}.conv.', cin_, cout))
    return s


def param_shapes(model_type, cfg):
    """Ordered {name: shape} matching the reference's named_parameters() order."""
    topo = list(cfg['TOPOLOGY'])
    cin, nout = cfg['IN_CHANNELS'], cfg['OUT_CHANNELS']
    n1, n2 = len(cfg['S1_BANDS']), len(cfg['S2_BANDS'])
    s = {}
    if model_type in ('siameseunet', 'unet', 'dtsiameseunet'):
        c = cin * 2 if model_type == 'unet' else cin
        s.update(_stream_shapes('inc.', 'encoder.', 'decoder.', c, topo))
        if model_type == 'dtsiameseunet':
            # module order: inc, encoder, decoder_change, decoder_sem, outc_change, outc_sem, outc_sem_change
            s = _stream_shapes('inc.', 'encoder.', 'decoder_change.', c, topo)
            s.update({k: v for k, v in _stream_shapes('inc.', 'encoder.', 'decoder_sem.', c, topo).items()
                      if k.startswith('decoder_sem.')})
            for h, ci, co in (('outc_change.', topo[0], nout), ('outc_sem.', topo[0], nout), ('outc_sem_change.', 2, 1)):
                s[h + 'conv.weight'] = (co, ci, 1, 1)
                s[h + 'conv.bias'] = (co,)
        else:
            s['outc.conv.weight'] = (nout, topo[0], 1, 1)
            s['outc.conv.bias'] = (nout,)
        return s
    if model_type == 'dualstreamunet':
        s.update(_stream_shapes('inc_stream1.', 'encoder_stream1.', 'decoder_stream1.', 2 * n1, topo))
        s.update(_stream_shapes('inc_stream2.', 'encoder_stream2.', 'decoder_stream2.', 2 * n2, topo))
        s['outc.conv.weight'] = (nout, 2 * topo[0], 1, 1)
        s['outc.conv.bias'] = (nout,)
        return s
    if model_type in ('whatevernet', 'whatevernet2'):
        for k, nb in ((1, n1), (2, n2)):
            nb = nb if model_type == 'whatevernet' else 2 * nb  # WhateverNet2: early fusion of t1 and t2 bands
            s.update(_stream_shapes(f'inc_stream{k}.', f'encoder_stream{k}.', f'decoder_stream{k}.', nb, topo))
            s[f'outc_stream{k}.conv.weight'] = (nout, topo[0], 1, 1)
            s[f'outc_stream{k}.conv.bias'] = (nout,)
        s['outc_fusion.conv.weight'] = (nout, 2 * topo[0], 1, 1)
        s['outc_fusion.conv.bias'] = (nout,)
        return s
    raise ValueError(model_type)


def bn_keys(shapes):
    """BatchNorm module prefixes (their weight is 1-D and sits at Sequential index 1 or 4)."""
    return [k[:-len('.weight')] for k, v in shapes.items()
            if k.endswith('.weight') and len(v) == 1 and (k.endswith('conv.1.weight') or k.endswith('conv.4.weight'))]


def deterministic_params(shapes, seed):
    """Seeded bounded fill: conv weights U(-1,1)/sqrt(fan_in); biases U(-0.1, 0.1); BN gamma 1+U(-.1,.1), beta U(-.1,.1)."""
    import numpy as np

    rng = np.random.default_rng(seed)
    P = {}
    for k, shp in shapes.items():
        u = rng.uniform(-1.0, 1.0, size=shp).astype(np.float32)
        if len(shp) == 4:
            fan_in = shp[1] * shp[2] * shp[3]
            v = u / np.sqrt(fan_in)
        elif k.endswith('conv.1.weight') or k.endswith('conv.4.weight'):
            v = 1.0 + 0.1 * u
        else:
            v = 0.1 * u
        P[k] = torch.from_numpy(np.ascontiguousarray(v, dtype=np.float32))
    return P


def fresh_buffers(shapes):
    B = {}
    for key in bn_keys(shapes):
        c = shapes[key + '.weight'][0]
        B[key + '.running_mean'] = torch.zeros(c)
        B[key + '.running_var'] = torch.ones(c)
        B[key + '.num_batches_tracked'] = torch.zeros((), dtype=torch.long)
    return B


def synthetic_batch(cfg, batch, hw, seed, labeled=None):
    """Seeded synthetic item-dict batch (utils/datasets.py:164-179 contract)."""
    import numpy as np

    rng = np.random.default_rng(seed)
    c = cfg['IN_CHANNELS']
    h, w = (hw, hw) if isinstance(hw, int) else tuple(hw)
    f = lambda *s: torch.from_numpy(rng.random(s, dtype=np.float32))
    out = {
        'x_t1': f(batch, c, h, w),
        'x_t2': f(batch, c, h, w),
        'y_change': (f(batch, 1, h, w) > 0.9).float(),
        'y_sem_t1': (f(batch, 1, h, w) > 0.8).float(),
        'y_sem_t2': (f(batch, 1, h, w) > 0.8).float(),
    }
    out['is_labeled'] = torch.tensor(labeled if labeled is not None else [True] * batch)
    return out
