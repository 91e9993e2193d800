"""Stage executors of the Siamese U-Net hot path: torch.autograd.Functions over libscd (HIP, gfx950).

Each Function runs a whole stage of the reference's forward (utils/networks.py) as a sequence of C-ABI
calls on NHWC fp32 device buffers, and its backward as the reverse sequence:

  pack_pair / pack_stream  input NCHW -> NHWC (+ channel padding)        train_supervised.py:68-69
  EncoderLevelFn           one level of InConv + Encoder (Down x L)       networks.py:313-343, 405-426
  SiameseLevelFn           the same on the t1/t2 pair batch, + f_t2 - f_t1 networks.py:141-150
  SiameseDiffFn            f_t2 - f_t1                                     networks.py:147-150
  DecoderFn                Up x L (ConvT -> cat -> DoubleConv)             networks.py:346-382, 429-451
  HeadFn                   OutConv 1x1                                     networks.py:454-461
  CatFn                    torch.cat(..., dim=1) of decoder outputs        networks.py:119, 258
  PJaccardFn               power_jaccard_loss                              loss_functions.py:141-150

The Siamese encoder runs both branches as ONE 2B-image batch (weights shared) with BatchNorm
statistics segmented per branch (nseg = 2), which reproduces the reference's two separate module calls
exactly: per-branch batch statistics, two running-stat updates (t1 first), summed weight grads.
"""
from __future__ import annotations

import contextlib
import contextvars
import weakref
from dataclasses import dataclass

import torch

from . import hip
from .hip import TAPS_1, TAPS_2X2, TAPS_3X3, nhwc

_F32 = torch.float32

# Fusion switches (tools/ab_step.py flips them for in-process A/B; results are identical either way).
_OPTS = {'fuse_input_bn': True, 'fuse_bn_bwd': True, 'fuse_siamese_encoder': True, 'batch_pack': True,
         'pack_cache': True, 'pool_diff': True, 'pooled_bn_bwd': True, 'defer_bn_bwd': True, 'fuse_head': True,
         'convT_bias_in_wgrad': True, 'head_wgrad_in_bn_bwd': True, 'fuse_plain_encoder': True,
         'fuse_dualtask': True, 'dt_sem_batched': True, 'fuse_heads': True, 'bn_bwd_in_wgrad': 128}
# bn_bwd_in_wgrad: the widest weight-grad source (channels) whose conv's plain BatchNorm backward is formed inside the
# weight grad (0 = never).  Wider sources are split over more 64-channel tiles that each read the rows again, and
# reading y and da instead of dy there cost more than the apply pass saved.  Same-process A/B
# (profiles/r05_bn_bwd_in_wgrad_ab.txt): Siamese bs=32 off 30.05, <= 64 30.02, <= 128 29.81 ms; dual-stream bs=64 off
# 41.89, <= 64 41.62, <= 128 41.63 ms, no limit 42.30 (vs 41.80 off).


def conv_math_for(cfg) -> str:
    """The conv arithmetic a config asks for: MODEL.CONV_MATH if set, else MODEL.PRECISION ('fp32' -> the
    fp32-accurate two-term fp16 split 'h2' (bounded operands; every other conv runs the split-bf16 'x3'),
    'bf16' -> 'bf16')."""
    m = cfg.MODEL.get('CONV_MATH', None)
    if m:
        return str(m)
    prec = str(cfg.MODEL.get('PRECISION', 'fp32')).lower()
    if prec in ('bf16', 'bfloat16'):
        return 'bf16'
    if prec in ('fp32', 'f32', 'float32'):
        return 'h2'
    raise ValueError(f"MODEL.PRECISION {prec!r}: expected 'fp32' or 'bf16'")


def option(name: str):
    return _OPTS[name]


def set_options(**kw) -> dict:
    """fuse_input_bn: apply a DoubleConv's first BatchNorm + ReLU inside the second conv's operand staging
    (forward and weight-grad) instead of materialising the activation.
    fuse_bn_bwd: compute the first BatchNorm's backward partial sums in the epilogue of the data-grad conv that
    produces its incoming gradient, instead of a separate pass.
    fuse_siamese_encoder: Siamese streams run SiameseLevelFn (BN1 + ReLU fused into the next MaxPool and the
    feature difference, differences written into the decoder's concat buffers).
    defer_bn_bwd: the input layer's BatchNorm backward stops at its statistics and the weight grad (its only
    reader) forms dy while staging, so that gradient is never written.
    fuse_head: a 1x1 head that is a decoder output's only reader runs inside the decoder stage (run_decoder head=),
    reading the last BatchNorm + ReLU through its coefficients.
    fuse_plain_encoder: a plain (non-Siamese) encoder level writes its activation straight into the decoder's concat
    buffer and pools it in the same pass (scd_bn_relu_pool_out mode 1): no bn_relu_apply, no skip copy.
    fuse_dualtask: DualTaskSiameseUNet's encoder levels write the difference (decoder_change) and the [t2; t1] skip
    batch (decoder_sem) in one pass (mode 2), the encoder backward forms both skip gradients on the fly.
    dt_sem_batched: decoder_sem runs both dates as ONE 2B-image batch with per-date BatchNorm segments (t2 first)
    instead of two calls (same per-call statistics and running-stat order; weight grads summed in another order).
    fuse_heads: the two-decoder models' heads (DualStream's outc, WhateverNet(2)'s outc_stream1/2 + outc_fusion) run as
    one launch over both decoders' last BatchNorm + ReLU (no cat, no materialised decoder outputs).
    bn_bwd_in_wgrad (int, channels): a plain BatchNorm backward whose conv's weight-grad source has at most this many
    channels is formed inside that weight grad, which also stores dy for the data grad (ABI 8): no apply pass; 0 = off.
    Returns the previous options."""
    prev = dict(_OPTS)
    for k, v in kw.items():
        if k not in _OPTS:
            raise KeyError(k)
        _OPTS[k] = v
    return prev


# ------------------------------------------------------------------------------------------------
# Conv weight preparation, batched per step.  Every 3x3 conv weight of a model is registered with its model's
# group (register_weight_group, called by create_network).  The first packed-layout request of a forward pass
# packs (and bf16x3-splits) the whole group in ONE scd_pack_conv3x3_multi launch; later requests of that
# forward and its backward hit the cache.  A forward pre-hook on the model starts a new generation, so weights
# are repacked once per forward pass whatever changed them (optimizers do not reliably bump parameter version
# counters: torch's fused AdamW does not).  Weights outside a registered model are packed on every call.
# ------------------------------------------------------------------------------------------------
class _IdentityMap:
    """Tensor-keyed map by object identity (tensor == is elementwise), dropping entries when the key dies."""

    def __init__(self):
        self._d = {}

    def get(self, t):
        ent = self._d.get(id(t))
        return ent[1] if ent is not None and ent[0]() is t else None

    def setdefault(self, t, value):
        v = self.get(t)
        if v is None:
            k = id(t)
            self._d[k] = (weakref.ref(t, lambda _r, k=k, d=self._d: d.pop(k, None)), value)
            v = value
        return v

    def clear(self):
        self._d.clear()


class _WeightGroup:
    def __init__(self, weights, convT_weights=()):
        self.refs = [weakref.ref(w) for w in weights]  # 3x3 conv weights
        self.trefs = [weakref.ref(w) for w in convT_weights]  # ConvTranspose2d(2, s2) weights
        self.gen = 0


_GROUPS = _IdentityMap()  # weight Parameter -> its model's _WeightGroup
_PACKED = _IdentityMap()  # weight Parameter -> {key: (generation, data_ptr, packed tensor)}


def register_weight_group(model: torch.nn.Module):
    convs = [m for m in model.modules() if isinstance(m, torch.nn.Conv2d) and m.kernel_size == (3, 3)]
    convTs = [m for m in model.modules() if isinstance(m, torch.nn.ConvTranspose2d) and m.kernel_size == (2, 2)]
    group = _WeightGroup([c.weight for c in convs], [c.weight for c in convTs])
    for c in convs + convTs:
        _GROUPS.setdefault(c.weight, group)

    def new_generation(_module, _args):
        group.gen += 1

    model.register_forward_pre_hook(new_generation)


def invalidate_weight_cache():
    _PACKED.clear()


def _pack_key(mode: int, ci_pad: int):
    return (mode, ci_pad if mode == 0 else 0, hip.conv_math())


def _cached(w, key, group):
    ent = (_PACKED.get(w) or {}).get(key)
    if ent is not None and ent[0] == group.gen and ent[1] == w.data_ptr():
        return ent[2]
    return None


def packed_conv3x3(weight: torch.Tensor, mode: int, ci_pad: int | None = None) -> torch.Tensor:
    """hip.pack_conv3x3(weight, mode, ci_pad) through the per-forward group cache."""
    ci_pad = weight.shape[1] if ci_pad is None else ci_pad
    group = _GROUPS.get(weight)
    if not _OPTS['pack_cache'] or group is None:
        return hip.pack_conv3x3(weight.detach(), mode, ci_pad=ci_pad if mode == 0 else None)
    key = _pack_key(mode, ci_pad)
    hit = _cached(weight, key, group)
    if hit is not None:
        return hit
    todo = [(weight, ci_pad)]
    if _OPTS['batch_pack']:
        for r in group.refs:
            w = r()
            if w is None or w is weight or w.device != weight.device:
                continue
            cp = pad_in(w.shape[1]) if mode == 0 else w.shape[1]
            if mode == 1 and w.shape[1] % 8:  # input-layer convs: no data grad is ever taken
                continue
            if _cached(w, _pack_key(mode, cp), group) is None:
                todo.append((w, cp))
    with torch.no_grad():
        packs = hip.pack_conv3x3_multi([(w.detach(), mode, cp) for w, cp in todo])
    for (w, cp), pk in zip(todo, packs):
        _PACKED.setdefault(w, {})[_pack_key(mode, cp)] = (group.gen, w.data_ptr(), pk)
    return packs[0]


def packed_convT2x2(weight: torch.Tensor, mode: int) -> torch.Tensor:
    """hip.pack_convT2x2(weight, mode) through the per-forward group cache: the first request of a forward packs (and
    splits) every ConvTranspose weight of the model in that layout in one batched call (scd_pack_convT2x2_multi)."""
    group = _GROUPS.get(weight)
    if not _OPTS['pack_cache'] or group is None or not any(r() is weight for r in group.trefs):
        return hip.pack_convT2x2(weight.detach(), mode)
    key = ('convT', mode, hip.conv_math())
    hit = _cached(weight, key, group)
    if hit is not None:
        return hit
    todo = [weight]
    if _OPTS['batch_pack']:
        for r in group.trefs:
            w = r()
            if w is not None and w is not weight and w.device == weight.device and _cached(w, key, group) is None:
                todo.append(w)
    with torch.no_grad():
        packs = hip.pack_convT2x2_multi([(w.detach(), mode) for w in todo])
    for w, pk in zip(todo, packs):
        _PACKED.setdefault(w, {})[key] = (group.gen, w.data_ptr(), pk)
    return packs[0]


def _empty(shape, like: torch.Tensor, dtype=_F32):
    return torch.empty(shape, device=like.device, dtype=dtype)


def _act(shape, like: torch.Tensor):
    """An activation / gradient buffer in the storage type of `like` (fp32, or bf16 under bf16 storage)."""
    return torch.empty(shape, device=like.device, dtype=like.dtype)


# Activation and gradient storage of the model being run (act_storage_for / storage_scope): the input packing creates
# its NHWC tensors in this type, and every buffer downstream inherits the type of the activation it derives from.
_STORAGE = contextvars.ContextVar('scd_act_storage', default=_F32)


@contextlib.contextmanager
def storage_scope(dtype):
    tok = _STORAGE.set(dtype)
    try:
        yield
    finally:
        _STORAGE.reset(tok)


def act_storage_for(cfg, math: str | None = None):
    """torch dtype of a model's activations and gradients in HBM: bf16 for the bf16 arithmetic when every conv of the
    model has a bf16-storage kernel (TOPOLOGY channel counts multiples of 64, padded input widths 16 or a multiple of
    64 (input_widths): the bf16 halo16, c16, gather16 and ConvTranspose weight-grad kernels), else fp32.  MODEL.ACT_STORAGE ('fp32' / 'bf16') overrides."""
    math = math or conv_math_for(cfg)
    want = str(cfg.MODEL.get('ACT_STORAGE', '') or '').lower()
    if want in ('fp32', 'f32', 'float32'):
        return _F32
    ok = (math == 'bf16' and all(int(c) % 64 == 0 for c in cfg.MODEL.TOPOLOGY)
          and all(w == 16 or w % 64 == 0 for w in input_widths(cfg)))
    if want in ('bf16', 'bfloat16'):
        if not ok:
            raise ValueError("MODEL.ACT_STORAGE bf16 needs MODEL.PRECISION bf16, TOPOLOGY channels in multiples of 64 "
                             f"and padded input widths of 16 or multiples of 64 (got {input_widths(cfg)})")
        return torch.bfloat16
    if want:
        raise ValueError(f"MODEL.ACT_STORAGE {want!r}: expected 'fp32' or 'bf16'")
    return torch.bfloat16 if ok else _F32


def input_widths(cfg) -> list:
    """The channel widths a model's input layers see under the bf16 arithmetic (bands padded to the 16-channel
    granule, pad_in): pack_pair of IN_CHANNELS (Siamese, dual-task), pack_stream of both dates' bands (UNet,
    DualStream, WhateverNet2), pack_pair per modality (WhateverNet)."""
    def p16(c):
        return (int(c) + 15) // 16 * 16
    t = str(cfg.MODEL.TYPE)
    if t in ('dualstreamunet', 'whatevernet', 'whatevernet2'):
        n1, n2 = len(cfg.DATALOADER.S1_BANDS), len(cfg.DATALOADER.S2_BANDS)
        k = 1 if t == 'whatevernet' else 2
        return [p16(k * n1), p16(k * n2)]
    c = int(cfg.MODEL.IN_CHANNELS)
    return [p16(2 * c if t == 'unet' else c)]


def storage_for_input(dtype, h: int, w: int, levels: int):
    """The storage a forward on (h, w) tiles runs in: bf16 storage needs every level's map tiled by the bf16 kernels
    (the deepest, h / 2^(levels - 1), a multiple of 16 both ways); other tiles (e.g. full-AOI evaluation) run fp32."""
    if dtype == _F32:
        return _F32
    g = 16 << max(levels - 1, 0)
    return dtype if h % g == 0 and w % g == 0 else _F32


def _ws(nbytes: int, like: torch.Tensor):
    return torch.empty(int(nbytes), device=like.device, dtype=torch.uint8)


# ------------------------------------------------------------------------------------------------
# SCD_MATH_H2 operand bounds.  The h2 conv arithmetic scales each activation operand by the power of two of an
# upper bound of its magnitude (scd_igemm_t.src_bound).  The bounds come from the producers at no extra pass:
# a BatchNorm's statistics bound its ReLU output (scd_bn_*_stats act_bound), the BatchNorm backward raises a bound
# to max |dy| as it writes dy (dy_bound); scd_absmax_bound covers the rest (eval mode, the ConvT half of a concat).
# A bound is a one-float device tensor; bounds are only allocated under h2.
# ------------------------------------------------------------------------------------------------
_ARENA_FLOATS = 4096
_ZERO_ARENA: dict = {}  # device -> [zeroed float buffer, floats handed out]


def _zero_float(device) -> torch.Tensor:
    """A fresh zero-initialised device float, carved from a per-device arena: one fill launch per 4096 bounds
    instead of one per stage and input (~30 fills per training step before).  A float is never handed out twice."""
    ent = _ZERO_ARENA.get(device)
    if ent is None or ent[1] == _ARENA_FLOATS:
        ent = _ZERO_ARENA[device] = [torch.zeros(_ARENA_FLOATS, device=device, dtype=_F32), 0]
    ent[1] += 1
    return ent[0][ent[1] - 1:ent[1]]


class _Bounds:
    """Zero-initialised device floats handed out one at a time (from the per-device arena)."""

    def __init__(self, like: torch.Tensor):
        self.device = like.device

    def take(self) -> torch.Tensor:
        return _zero_float(self.device)


def _bounds(like: torch.Tensor):
    """A bound pool under the h2 arithmetic, else None (no bounds anywhere)."""
    return _Bounds(like) if hip.conv_math() == 'h2' else None


def _take(pool):
    return pool.take() if pool is not None else None


_ACT_BOUND = _IdentityMap()  # activation tensor handed between stages -> its bound


def _set_bound(t: torch.Tensor, b):
    if b is not None:
        _ACT_BOUND.setdefault(t, b)
    return t


def _bound_of(t: torch.Tensor, pool, nseg: int = 1, scale=None, shift=None):
    """The registered bound of t, or (under h2) a fresh one from a pass over t."""
    if pool is None:
        return None
    b = _ACT_BOUND.get(t)
    if b is None:
        b = pool.take()
        hip.absmax_bound(nhwc(t), b, nseg, scale, shift)
    return b


def pad8(c: int) -> int:
    return (c + 7) // 8 * 8


def pad_in(c: int) -> int:
    """Input channel padding: the MFMA K granule -- 16 under the split-bf16 arithmetic (so the input layer
    takes the halo x3 path with fused BatchNorm statistics), 8 under fp32 MFMA."""
    g = 16 if hip.conv_math() != 'f32' else 8
    return (c + g - 1) // g * g


# ------------------------------------------------------------------------------------------------
# BatchNorm + ReLU
# ------------------------------------------------------------------------------------------------
@dataclass
class _BNSaved:
    smean: torch.Tensor
    sinv: torch.Tensor
    scale: torch.Tensor
    shift: torch.Tensor
    nseg: int


# BatchNorm `num_batches_tracked` increments of one stage, applied in one foreach launch when the stage ends
# (flush_bn_counters) instead of one int64 add per layer.
_NBT_PENDING: list = []


def flush_bn_counters() -> None:
    if not _NBT_PENDING:
        return
    by_inc: dict = {}
    for t, inc in _NBT_PENDING:
        by_inc.setdefault(inc, []).append(t)
    _NBT_PENDING.clear()
    for inc, ts in by_inc.items():
        torch._foreach_add_(ts, inc)


# Instrumentation for the parity tests (tests/_parity.py BranchMatch): while trace_bn() is open, every BatchNorm
# forward appends (module, conv output y, scale, shift, nseg) -- the values the ReLU decisions fma(y, scale, shift)
# > 0 and the MaxPool2d argmaxes of this forward are taken from, so a CPU oracle can follow the same branches.
_BN_TRACE: list | None = None


@contextlib.contextmanager
def trace_bn():
    global _BN_TRACE
    prev, _BN_TRACE = _BN_TRACE, []
    try:
        yield _BN_TRACE
    finally:
        _BN_TRACE = prev


def _traced(bn, y: torch.Tensor, st: '_BNSaved') -> '_BNSaved':
    if _BN_TRACE is not None:
        _BN_TRACE.append((bn, y.detach().clone(), st.scale.clone(), st.shift.clone(), st.nseg))
    return st


def _bn_uses_batch_stats(bn: torch.nn.BatchNorm2d, training: bool) -> bool:
    return training or not bn.track_running_stats or bn.running_mean is None


def _bn_forward(y: torch.Tensor, bn: torch.nn.BatchNorm2d, nseg: int, training: bool, tiles=None,
                bound=None) -> _BNSaved:
    """Batch statistics (train) or running statistics (eval) -> per-segment scale/shift.

    `tiles` = (tile records, ntiles, pixels per tile) from the conv that produced y (fused statistics);
    without it the statistics are a separate pass over y.  `bound` (h2): a zeroed device float raised to a bound
    of the activation relu(BN(y)) -- from the statistics in train mode, by a pass over y in eval mode.
    """
    n, h, w, c = y.shape
    if _bn_uses_batch_stats(bn, training):
        smean, sinv, scale, shift = (_empty((nseg * c,), y) for _ in range(4))
        update = training and bn.track_running_stats and bn.running_mean is not None
        mom = bn.momentum if bn.momentum is not None else 0.1
        if update and bn.momentum is None:
            raise NotImplementedError("BatchNorm2d(momentum=None) cumulative averaging is not supported")
        if tiles is not None:
            rec, ntiles, tpx = tiles
            ws = _ws(hip.bn_tile_stats_workspace_bytes(ntiles, c, nseg), y)
            hip.bn_stats_from_tiles(rec, ntiles, tpx, c, nseg, bn.weight, bn.bias, bn.eps, mom, update,
                                    bn.running_mean, bn.running_var, smean, sinv, scale, shift, ws, act_bound=bound)
        else:
            ws = _ws(hip.bn_workspace_bytes(n, h, w, c, nseg), y)
            hip.bn_train_stats(nhwc(y), nseg, bn.weight, bn.bias, bn.eps, mom, update, bn.running_mean,
                               bn.running_var, smean, sinv, scale, shift, ws, act_bound=bound)
        if update:
            _NBT_PENDING.append((bn.num_batches_tracked, nseg))
        return _traced(bn, y, _BNSaved(smean, sinv, scale, shift, nseg))
    scale, shift = _empty((c,), y), _empty((c,), y)
    hip.bn_eval_coeffs(c, bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.eps, scale, shift)
    if bound is not None:
        hip.absmax_bound(nhwc(y), bound, 1, scale, shift)
    return _traced(bn, y, _BNSaved(None, None, scale, shift, 1))


# ------------------------------------------------------------------------------------------------
# DoubleConv (networks.py:386-402): (conv3x3 -> BN -> ReLU) x 2
# ------------------------------------------------------------------------------------------------
def dc_params(dc) -> list:
    s = dc.conv
    return [s[0].weight, s[0].bias, s[1].weight, s[1].bias, s[3].weight, s[3].bias, s[4].weight, s[4].bias]


def _conv3x3_stats(x: torch.Tensor, wpk: torch.Tensor, bias, n_out: int, want: bool, in_bn=None, y=None,
                   src_bound=None):
    """Conv 3x3 forward; with `want`, also the fused per-tile BatchNorm statistics when the conv provides them.
    `in_bn` = (scale, shift, nseg): x is the previous conv's output, read through its BatchNorm + ReLU.
    `src_bound` (h2): the bound of x as read."""
    n, h, w, _ = x.shape
    y = _act((n, h, w, n_out), x) if y is None else y
    tiles = None
    if want:
        ntiles, tpx = hip.igemm_stat_tiles(nhwc(x), h, w, 1, TAPS_3X3, wpk, n_out, nhwc(y), src_bound=src_bound)
        if ntiles:
            rec = _empty((ntiles * n_out * 2,), x)
            tiles = (rec, ntiles, tpx)
    hip.conv_igemm(nhwc(x), h, w, 1, TAPS_3X3, wpk, n_out, bias, nhwc(y),
                   stat_rec=None if tiles is None else tiles[0], in_bn=in_bn, src_bound=src_bound)
    return y, tiles


def _can_fuse_input_bn(y0: torch.Tensor, wpk1: torch.Tensor, y1: torch.Tensor, st: '_BNSaved', save: bool,
                       bound=None) -> bool:
    """Whether conv1 (and, when training, its weight grad) can read y0 through BN0 + ReLU directly."""
    if not _OPTS['fuse_input_bn']:
        return False
    n, h, w, _ = y0.shape
    bn = (st.scale, st.shift, st.nseg)
    if not hip.igemm_input_bn_supported(nhwc(y0), h, w, 1, TAPS_3X3, wpk1, y1.shape[3], nhwc(y1), bn, bound):
        return False
    return not save or hip.wgrad_src_bn_supported(nhwc(y1), nhwc(y0), 1, TAPS_3X3, bn)


def _dc_forward(x: torch.Tensor, dc, nseg: int, training: bool, save: bool, materialize: bool = True,
                pool=None, x_bound=None):
    """(a1, saved, y1, st1, b1); with materialize=False the output activation a1 = relu(BN1(y1)) is left to the
    consumers (None is returned for it).  Under h2 (`pool` given) `x_bound` bounds x and b1 bounds a1."""
    s = dc.conv
    conv0, bn0, conv1, bn1 = s[0], s[1], s[3], s[4]
    cin = x.shape[3]
    if conv0.in_channels > cin:
        raise ValueError(f"DoubleConv expects {conv0.in_channels} input channels, got {cin}")
    if pool is not None and x_bound is None and (cin % 32 == 0 or cin == 16):
        x_bound = _bound_of(x, pool)  # the 16-channel input layer: the packing's bound (igemm_halo16_c16 h2)
    y0, t0 = _conv3x3_stats(x, packed_conv3x3(conv0.weight, 0, ci_pad=cin), conv0.bias,
                            conv0.out_channels, _bn_uses_batch_stats(bn0, training), src_bound=x_bound)
    b0 = _take(pool)
    st0 = _bn_forward(y0, bn0, nseg, training, t0, b0)
    wpk1 = packed_conv3x3(conv1.weight, 0)
    n, h, w, _ = y0.shape
    y1 = _act((n, h, w, conv1.out_channels), y0)
    if _can_fuse_input_bn(y0, wpk1, y1, st0, save, b0):
        a0 = None  # never materialised: conv1 and its weight grad apply BN0 + ReLU while staging y0
        y1, t1 = _conv3x3_stats(y0, wpk1, conv1.bias, conv1.out_channels, _bn_uses_batch_stats(bn1, training),
                                in_bn=(st0.scale, st0.shift, st0.nseg), y=y1, src_bound=b0)
    else:
        a0 = torch.empty_like(y0)
        hip.bn_relu_apply(nhwc(y0), st0.nseg, st0.scale, st0.shift, nhwc(a0))
        y1, t1 = _conv3x3_stats(a0, wpk1, conv1.bias, conv1.out_channels, _bn_uses_batch_stats(bn1, training), y=y1,
                                src_bound=b0)
    b1 = _take(pool)
    st1 = _bn_forward(y1, bn1, nseg, training, t1, b1)
    a1 = None
    if materialize:
        a1 = torch.empty_like(y1)
        hip.bn_relu_apply(nhwc(y1), st1.nseg, st1.scale, st1.shift, nhwc(a1))
        _set_bound(a1, b1)
    saved = (x, y0, a0, st0, y1, st1, x_bound, b0) if save else None
    return a1, saved, y1, st1, b1


def _wgrad3x3(dy: torch.Tensor, x: torch.Tensor, weight: torch.Tensor, src_bn=None, rows_bound=None,
              src_bound=None, rows_bn=None, rows_out=None, rows_out_bound=None) -> torch.Tensor:
    """`rows_bn` (hip._rows_bn_fields): dy is dL/da, formed into the BatchNorm backward's dy while staging;
    `rows_out` then receives that dy (and `rows_out_bound` its max |dy|) for the data grad."""
    if rows_bound is None or src_bound is None:
        rows_bound = src_bound = None
    d, nsplit, nbytes = hip.wgrad_plan(nhwc(dy), nhwc(x), 1, TAPS_3X3, src_bn, rows_bound, src_bound, rows_bn,
                                       None if rows_out is None else nhwc(rows_out), rows_out_bound)
    slabs = _empty((nbytes // 4,), dy)
    hip.conv_wgrad(d, slabs)
    gw = torch.empty_like(weight)
    hip.wgrad_finalize(slabs, nsplit, dy.shape[3], 9, x.shape[3], 0, weight.shape[1], gw)
    return gw


@dataclass
class _PooledGrad:
    """An encoder level's incoming gradient, maxpool_bwd(gy, idx) -/+ gskip, left unmaterialised: the BatchNorm
    backward forms it on the fly (scd_bn_relu_backward_pooled)."""
    gy: torch.Tensor | None
    idx: torch.Tensor | None
    gskip: torch.Tensor | None
    skip_mode: int
    gskip2: torch.Tensor | None = None  # skip_mode 2: the dual-task semantic skip gradient, [t2; t1]


@dataclass
class _HeadGrad:
    """The decoder's last gradient when the 1x1 head reads its output through the BatchNorm + ReLU: dL/da =
    g . w2 (g: the logits' gradient, NCHW; w2: [n_out][C]), formed inside the BatchNorm backward
    (scd_bn_relu_backward_head) instead of being written by the head's backward."""
    g: torch.Tensor
    w2: torch.Tensor
    n_out: int
    w_grad: torch.Tensor | None = None  # also the head's weight grad ([n_out][C]) from the same pass


def _bn_backward(y, g, st: _BNSaved, bn, conv_bias_grad: bool, tiles=None, dy_bound=None):
    """`tiles` = (records, ntiles) of the partial sums from the conv epilogue that produced g; g may be a
    _PooledGrad.  `dy_bound` (h2): a zeroed device float raised to max |dy|."""
    c = y.shape[3]
    dy = torch.empty_like(y)
    dgamma = _empty((c,), y)
    dbeta = _empty((c,), y)
    dbias = _empty((c,), y) if conv_bias_grad else None
    n, h, w, _ = y.shape
    ws = _ws(hip.bn_workspace_bytes(n, h, w, c, st.nseg), y)
    if isinstance(g, _HeadGrad):
        if g.w_grad is not None:
            ws = _ws(hip.bn_head_workspace_bytes(n, h, w, c, st.nseg, g.n_out), y)
        hip.bn_relu_backward_head(nhwc(y), g.g, g.w2, g.n_out, st.nseg, st.smean, st.sinv, bn.weight, st.scale,
                                  st.shift, dgamma, dbeta, dbias, nhwc(dy), ws, dy_bound, g.w_grad)
    elif isinstance(g, _PooledGrad) and g.gskip2 is not None:
        hip.bn_relu_backward_pooled2(nhwc(y), nhwc(g.gy) if g.gy is not None else hip._NULL, g.idx, nhwc(g.gskip),
                                     g.skip_mode, nhwc(g.gskip2), st.nseg, st.smean, st.sinv, bn.weight, st.scale,
                                     st.shift, dgamma, dbeta, dbias, nhwc(dy), ws, dy_bound)
    elif isinstance(g, _PooledGrad):
        hip.bn_relu_backward_pooled(nhwc(y), nhwc(g.gy) if g.gy is not None else hip._NULL, g.idx,
                                    nhwc(g.gskip) if g.gskip is not None else hip._NULL, g.skip_mode, st.nseg,
                                    st.smean, st.sinv, bn.weight, st.scale, st.shift, dgamma, dbeta, dbias, nhwc(dy),
                                    ws, dy_bound)
    elif tiles is not None:
        hip.bn_relu_backward_tiles(nhwc(y), nhwc(g), st.nseg, st.smean, st.sinv, bn.weight, st.scale, st.shift,
                                   tiles[0], tiles[1], dgamma, dbeta, dbias, nhwc(dy), ws, dy_bound)
    else:
        hip.bn_relu_backward(nhwc(y), nhwc(g), st.nseg, st.smean, st.sinv, bn.weight, st.scale, st.shift, dgamma,
                             dbeta, dbias, nhwc(dy), ws, dy_bound)
    return dy, dgamma, dbeta, dbias


def _bn_backward_coef(y, g, st: _BNSaved, bn, conv_bias_grad: bool, tiles=None, da_bound=None, dy_bound=None):
    """The statistics half of _bn_backward (hip.bn_relu_backward_coef): (dgamma, dbeta, dbias, coef).  `dy_bound`
    (h2, with `da_bound` bounding g): a zeroed device float raised to a bound of the dy the consumer forms."""
    c = y.shape[3]
    dgamma, dbeta = _empty((c,), y), _empty((c,), y)
    dbias = _empty((c,), y) if conv_bias_grad else None
    coef = _empty((st.nseg * c * 2,), y)
    n, h, w, _ = y.shape
    ws = _ws(hip.bn_workspace_bytes(n, h, w, c, st.nseg), y)
    hip.bn_relu_backward_coef(nhwc(y), nhwc(g), st.nseg, st.smean, st.sinv, bn.weight, st.scale, st.shift,
                              tiles[0] if tiles is not None else None, tiles[1] if tiles is not None else 0, coef,
                              dgamma, dbeta, dbias, ws, da_bound, dy_bound)
    return dgamma, dbeta, dbias, coef


def _dgrad_bn_bwd(dy1: torch.Tensor, wpk: torch.Tensor, n_out: int, y0: torch.Tensor, st0: _BNSaved,
                  src_bound=None, pool=None):
    """Data-grad conv producing dL/da0, with BN0's backward partial sums fused into its epilogue when the kernel
    offers them.  Returns (ga0, tiles or None, bound of ga0 or None).  `pool` (h2): the epilogue also raises a bound
    of ga0 where the kernel runs h2 (for a consumer that forms BN0's dy itself, _bn_backward_coef)."""
    n, h, w, _ = dy1.shape
    ga0 = _act((n, h, w, n_out), dy1)
    gb = None
    if pool is not None and hip.igemm_arith(nhwc(dy1), h, w, 1, TAPS_3X3, wpk, n_out, nhwc(ga0),
                                            src_bound=src_bound) == 'h2':
        gb = pool.take()
    if _OPTS['fuse_bn_bwd'] and st0.smean is not None:
        ntiles, _ = hip.igemm_bn_bwd_tiles(nhwc(dy1), h, w, 1, TAPS_3X3, wpk, n_out, nhwc(ga0), src_bound)
        if ntiles and ntiles % st0.nseg == 0:
            rec = _empty((n_out * ntiles * 2,), dy1)
            hip.conv_igemm(nhwc(dy1), h, w, 1, TAPS_3X3, wpk, n_out, None, nhwc(ga0),
                           bn_bwd=(y0, st0.nseg, st0.smean, st0.sinv, st0.scale, st0.shift, rec), src_bound=src_bound,
                           dst_bound=gb)
            return ga0, (rec, ntiles), gb
    hip.conv_igemm(nhwc(dy1), h, w, 1, TAPS_3X3, wpk, n_out, None, nhwc(ga0), src_bound=src_bound, dst_bound=gb)
    return ga0, None, gb


def _bn_backward_in_wgrad(y, g, st: _BNSaved, bn, conv, x, src_bn, x_bound, tiles, g_bound, pool):
    """A plain BatchNorm backward whose dy is read by this conv's weight grad and then its data grad: the weight grad
    forms dy while staging and stores it (scd_wgrad_t.rows_y / rows_out), so no apply pass runs.  Returns (dy, dgamma,
    dbeta, dbias, weight grad, bound of dy) or None where the kernels do not take it (the caller then runs
    _bn_backward).  Under h2 the weight grad scales dy by a bound from the statistics (_bn_backward_coef, needs
    g_bound) and raises the exact max |dy| for the data grad."""
    if not isinstance(g, torch.Tensor) or x.shape[3] > _OPTS['bn_bwd_in_wgrad'] or st.nseg > 2 or st.smean is None:
        return None
    if pool is not None and (g_bound is None or x_bound is None):
        return None
    rb = pool.take() if pool is not None else None
    if not hip.wgrad_rows_bn_supported(nhwc(g), nhwc(x), 1, TAPS_3X3, src_bn, rb, x_bound if rb is not None else None):
        return None
    dg, db, dbias, coef = _bn_backward_coef(y, g, st, bn, conv.bias is not None, tiles, g_bound, rb)
    dy = torch.empty_like(y)
    ob = pool.take() if pool is not None else None
    rows_bn = (nhwc(y), st.nseg, st.smean, st.sinv, bn.weight, st.scale, st.shift, coef)
    gw = _wgrad3x3(g, x, conv.weight, src_bn, rb, x_bound, rows_bn, rows_out=dy, rows_out_bound=ob)
    return dy, dg, db, dbias, gw, ob


def _dc_backward(g_out, saved, dc, need_dx: bool, pool=None, dy1_given: bool = False):
    """g_out: gradient of the block output (a tensor, or a _PooledGrad formed inside the BatchNorm backward).
    Returns (grad wrt DoubleConv input or None, [8 param grads in dc_params order]).  `pool` (h2): bounds of the
    two BatchNorm-backward outputs, the operands of the data-grad and weight-grad convs.
    dy1_given: g_out is already the gradient of the second conv's output y1 (its BatchNorm backward ran in the heads'
    backward, HeadsFn); that BatchNorm's and conv bias's gradients are then None here."""
    x, y0, a0, st0, y1, st1, x_bound, b0 = saved
    s = dc.conv
    conv0, bn0, conv1, bn1 = s[0], s[1], s[3], s[4]
    if st1.smean is None:
        raise RuntimeError("backward through an eval-mode BatchNorm is not supported (call net.train())")
    src_bn1 = (st0.scale, st0.shift, st0.nseg) if a0 is None else None  # fused forward: y0 through BN0 + ReLU
    x1 = y0 if a0 is None else a0
    fused1 = None
    if dy1_given:
        dy1, dg1, db1, dbias1 = g_out, None, None, None
        d1 = _bound_of(dy1, pool)
    else:
        fused1 = _bn_backward_in_wgrad(y1, g_out, st1, bn1, conv1, x1, src_bn1, b0, None,
                                       _ACT_BOUND.get(g_out) if pool is not None and isinstance(g_out, torch.Tensor)
                                       else None, pool)
        if fused1 is not None:
            dy1, dg1, db1, dbias1, gw1, d1 = fused1
        else:
            d1 = _take(pool)
            dy1, dg1, db1, dbias1 = _bn_backward(y1, g_out, st1, bn1, conv1.bias is not None, dy_bound=d1)
    if fused1 is None:
        gw1 = _wgrad3x3(dy1, x1, conv1.weight, src_bn1, d1, b0)
    # the bound of ga0 (h2), only for a weight grad that forms BN0's dy itself: the input layer's (deferred) or one
    # _bn_backward_in_wgrad can take (its source width and segment count; it still checks the kernel's shape)
    bwd_in_wgrad0 = need_dx and x.shape[3] <= _OPTS['bn_bwd_in_wgrad'] and st0.nseg <= 2 and st0.smean is not None
    ga0, tiles0, gb0 = _dgrad_bn_bwd(dy1, packed_conv3x3(conv1.weight, 1), conv1.in_channels, y0, st0, d1,
                                     pool if not need_dx or bwd_in_wgrad0 else None)
    if not need_dx and _OPTS['defer_bn_bwd'] and hip.wgrad_rows_bn_supported(nhwc(ga0), nhwc(x), 1, TAPS_3X3):
        # the input layer: dy0 has one reader, the weight grad, which forms it while staging; under h2 its bound
        # comes from the statistics and the bound of ga0 (the h2 input-layer weight grad)
        rb0 = _take(pool) if gb0 is not None and x_bound is not None else None
        dg0, db0, dbias0, coef = _bn_backward_coef(y0, ga0, st0, bn0, conv0.bias is not None, tiles0,
                                                   gb0 if rb0 is not None else None, rb0)
        rows_bn = (nhwc(y0), st0.nseg, st0.smean, st0.sinv, bn0.weight, st0.scale, st0.shift, coef)
        gw0 = _wgrad3x3(ga0, x, conv0.weight, None, rb0, x_bound, rows_bn)
        return None, [gw0, dbias0, dg0, db0, gw1, dbias1, dg1, db1]
    fused0 = _bn_backward_in_wgrad(y0, ga0, st0, bn0, conv0, x, None, x_bound, tiles0, gb0, pool) if need_dx else None
    if fused0 is not None:
        dy0, dg0, db0, dbias0, gw0, d0 = fused0
    else:
        d0 = _take(pool)
        dy0, dg0, db0, dbias0 = _bn_backward(y0, ga0, st0, bn0, conv0.bias is not None, tiles0, d0)
        if pool is not None and x_bound is None and \
                hip.wgrad_arith(hip.wgrad_desc(nhwc(dy0), nhwc(x), 1, TAPS_3X3, None, d0, d0)) == 'h2':
            # a source the forward left unbounded (the channel-padded input layer, whose forward kernel is x3):
            # bounded here, where that puts its weight grad (the generic kernel) on h2
            x_bound = _bound_of(x, pool)
        gw0 = _wgrad3x3(dy0, x, conv0.weight, None, d0, x_bound)
    gx = None
    if need_dx:
        if x.shape[3] != conv0.in_channels:
            raise RuntimeError("input-gradient through a channel-padded first layer is not supported")
        n, h, w, _ = dy0.shape
        gx = _act((n, h, w, conv0.in_channels), dy0)
        wd = packed_conv3x3(conv0.weight, 1)
        # h2: the kernel raises gx's bound as it stores (the decoder's ConvT data grad reads gx through it)
        gxb = None
        if pool is not None and hip.igemm_arith(nhwc(dy0), h, w, 1, TAPS_3X3, wd, conv0.in_channels, nhwc(gx),
                                                src_bound=d0) == 'h2':
            gxb = pool.take()
        hip.conv_igemm(nhwc(dy0), h, w, 1, TAPS_3X3, wd, conv0.in_channels, None, nhwc(gx), src_bound=d0,
                       dst_bound=gxb)
        _set_bound(gx, gxb)
    return gx, [gw0, dbias0, dg0, db0, gw1, dbias1, dg1, db1]


# ------------------------------------------------------------------------------------------------
# Input packing
# ------------------------------------------------------------------------------------------------
def _check_input_pair(x_t1: torch.Tensor, x_t2: torch.Tensor) -> None:
    """Both inputs must be GPU tensors of one shape on one device: their data pointers go straight to a kernel."""
    hip.ensure_device(x_t1)
    hip.ensure_device(x_t2)
    if x_t1.dim() != 4 or x_t1.shape != x_t2.shape:
        raise ValueError(f"x_t1 and x_t2 must be (B, C, H, W) of one shape, got {tuple(x_t1.shape)} and "
                         f"{tuple(x_t2.shape)}")
    if x_t1.device != x_t2.device:
        raise ValueError(f"x_t1 is on {x_t1.device} but x_t2 is on {x_t2.device}")


def _input_bound(like: torch.Tensor):
    """Under h2, a zeroed device float the input packing raises to max |input| (the input layer's operand bound,
    registered for the packed tensor: no extra pass), else None."""
    return _zero_float(like.device) if hip.conv_math() == 'h2' else None


def pack_pair(x_t1: torch.Tensor, x_t2: torch.Tensor, c_begin: int = 0, c_count: int | None = None) -> torch.Tensor:
    """Siamese input: [2B, H, W, pad_in(C)] NHWC with t1 images first (one shared-encoder batch)."""
    _check_input_pair(x_t1, x_t2)
    if x_t1.requires_grad or x_t2.requires_grad:
        raise NotImplementedError("input gradients are not computed by the HIP path")
    b, c, h, w = x_t1.shape
    c_count = c - c_begin if c_count is None else c_count
    out = torch.empty((2 * b, h, w, pad_in(c_count)), device=x_t1.device, dtype=_STORAGE.get())
    bound = _input_bound(out)
    hip.pack_nchw(x_t1.float(), c_begin, c_count, out[:b], bound=bound)
    hip.pack_nchw(x_t2.float(), c_begin, c_count, out[b:], bound=bound)
    return _set_bound(out, bound)


def pack_stream(x_t1: torch.Tensor, x_t2: torch.Tensor, c_begin: int = 0, c_count: int | None = None) -> torch.Tensor:
    """Early-fusion input cat((t1[bands], t2[bands]), dim=1) as [B, H, W, pad_in(2*nb)] NHWC."""
    _check_input_pair(x_t1, x_t2)
    if x_t1.requires_grad or x_t2.requires_grad:
        raise NotImplementedError("input gradients are not computed by the HIP path")
    b, c, h, w = x_t1.shape
    c_count = c - c_begin if c_count is None else c_count
    cp = pad_in(2 * c_count)
    out = torch.empty((b, h, w, cp), device=x_t1.device, dtype=_STORAGE.get())
    # t1 bands -> channels [0, nb) (zero-padding the rest), then t2 bands -> [nb, 2nb)
    bound = _input_bound(out)
    hip.pack_nchw(x_t1.float(), c_begin, c_count, out, 0, cp, bound=bound)  # t1 bands -> [0, nb), zero-pad to cp
    hip.pack_nchw(x_t2.float(), c_begin, c_count, out, c_count, c_count, bound=bound)  # t2 bands -> [nb, 2nb)
    return _set_bound(out, bound)


# ------------------------------------------------------------------------------------------------
# Encoder: InConv + Down x L
# ------------------------------------------------------------------------------------------------
class _Meta:
    """Non-tensor arguments of a stage Function."""

    def __init__(self, **kw):
        self.__dict__.update(kw)


def encoder_blocks(inc, encoder) -> list:
    return [inc.conv] + [down.mpconv[1] for down in encoder.down_seq.values()]


# One autograd Function per encoder level (InConv = level 0, Down{k} = level k).  A level's parameter gradients are
# therefore final as soon as that level's backward returns -- the deepest level first -- and DDP can all-reduce them
# while the shallower levels' backward still runs (one Function for the whole encoder would hand every encoder
# gradient, 64% of the model's, to DDP only at the very end of the backward).  Each level also produces the next
# level's pooled input, so its backward receives the pooled gradient and the skip / difference gradient together and
# forms dL/da = maxpool_bwd(g_pool) +/- g_skip inside its BatchNorm backward (scd_bn_relu_backward_pooled).
def _level_grad(g_pool, idx, g_skip, skip_mode: int, like: torch.Tensor):
    """The incoming gradient of a level's output activation: a _PooledGrad formed inside the BatchNorm backward, or
    (engine option pooled_bn_bwd off) materialised by scd_feature_grad."""
    if _OPTS['pooled_bn_bwd'] and (g_pool is not None or g_skip is not None):
        return _PooledGrad(g_pool, idx if g_pool is not None else None, g_skip, skip_mode)
    ga = torch.empty_like(like)
    hip.feature_grad(nhwc(g_pool) if g_pool is not None else hip._NULL, idx if g_pool is not None else None,
                     nhwc(g_skip) if g_skip is not None else hip._NULL, skip_mode, nhwc(ga))
    return ga


def _even(h: int, w: int) -> bool:
    return h % 2 == 0 and w % 2 == 0 and h >= 2 and w >= 2


def _plain_level_out(y1, st1: _BNSaved, a, nxt, idx):
    """a = relu(BN1(y1)) (a may be the skip slice of a decoder concat buffer) and, if nxt is given, MaxPool2d(a) into
    nxt / idx: one pass over y1 for even maps (scd_bn_relu_pool_out mode 1), else apply + pool (bit-identical)."""
    _, h, w, _ = y1.shape
    if _even(h, w):
        hip.bn_relu_pool_out(nhwc(y1), st1.nseg, st1.scale, st1.shift, hip.POOL_COPY, hip._NULL, nhwc(a),
                             nhwc(nxt) if nxt is not None else hip._NULL, idx)
        return
    hip.bn_relu_apply(nhwc(y1), st1.nseg, st1.scale, st1.shift, nhwc(a))
    if nxt is not None:
        hip.maxpool2_fwd(nhwc(a), nhwc(nxt), idx)


class EncoderLevelFn(torch.autograd.Function):
    """One level of InConv + Encoder (networks.py:313-343, 405-426) on one BatchNorm-segmented batch: the level's
    DoubleConv output activation a (a decoder skip) and, below the deepest level, the next level's input MaxPool2d(a)
    with its argmax bytes.  meta.x_bound (h2) bounds the input; meta.out_bound receives a's.
    With the engine option fuse_plain_encoder, a is written by one pass over the conv output that also pools it, into
    channels [0, C) of the decoder's concat buffer when meta.extra names the Up's ConvT channels (zero-copy cat,
    networks.py:449; meta.buf is then that buffer)."""

    @staticmethod
    def forward(ctx, x, meta, *params):
        ctx.set_materialize_grads(False)
        meta.scope = (hip.conv_math(), hip.conv_tune())
        fused = _OPTS['fuse_plain_encoder']
        a, sv, y1, st1, bound = _dc_forward(x, meta.dc, meta.nseg, meta.training, meta.save, materialize=not fused,
                                            pool=meta.pool, x_bound=meta.x_bound)
        meta.out_bound = bound
        meta.buf = None
        n, h, w, c = y1.shape
        extra = getattr(meta, 'extra', 0)
        idx = nxt = None
        if not meta.last:
            nxt = _act((n, h // 2, w // 2, c), y1)
            idx = _empty((n, h // 2, w // 2, c), y1, dtype=torch.uint8)
        if fused:
            buf = _act((n, h, w, c + extra), y1)
            a = buf[..., :c] if extra else buf
            _plain_level_out(y1, st1, a, nxt, idx)  # the pooled map keeps the level's bound
            _set_bound(a, bound)
            meta.buf = buf if extra else None
        elif nxt is not None:
            hip.maxpool2_fwd(nhwc(a), nhwc(nxt), idx)
        outs = (a,) if nxt is None else (a, nxt)
        if meta.save:
            ctx.meta, ctx.saved = meta, (sv, idx)
        return outs

    @staticmethod
    def backward(ctx, g_a, g_next=None):
        meta = ctx.meta
        with hip.conv_scope(*meta.scope):
            sv, idx = ctx.saved
            ga = _level_grad(g_next, idx, g_a, 0, sv[4])
            gx, pg = _dc_backward(ga, sv, meta.dc, need_dx=ctx.needs_input_grad[0], pool=_bounds(sv[4]))
        ctx.saved = None
        return (gx, None, *pg)


def run_encoder(inc, encoder, x: torch.Tensor, nseg: int, training: bool, extra: dict | None = None,
                with_buffers: bool = False):
    """InConv + Encoder: the level activations, level 0 first (Encoder.forward returns them reversed).
    `extra` {level: ConvT channels} (decoder_cat_channels, engine option fuse_plain_encoder): each such level writes its
    activation into a decoder concat buffer; with_buffers=True returns (activations, buffers or None per level)."""
    blocks = encoder_blocks(inc, encoder)
    extra = extra if _OPTS['fuse_plain_encoder'] else None
    extra = extra or {}
    pool, bound = _bounds(x), None
    feats, bufs, cur = [], [], x
    try:
        for level, dc in enumerate(blocks):
            params = dc_params(dc)
            save = torch.is_grad_enabled() and (cur.requires_grad or any(p.requires_grad for p in params))
            meta = _Meta(dc=dc, nseg=nseg, training=training, save=save, last=level == len(blocks) - 1, pool=pool,
                         x_bound=bound, extra=extra.get(level, 0))
            outs = EncoderLevelFn.apply(cur, meta, *params)
            feats.append(outs[0])
            bufs.append(meta.buf)
            bound = meta.out_bound
            if not meta.last:
                cur = outs[1]
    finally:
        flush_bn_counters()
    return (feats, bufs) if with_buffers else feats


# ------------------------------------------------------------------------------------------------
# Dual-task Siamese encoder (DualTaskSiameseUNet, networks.py:176-197): every level activation of both dates feeds the
# difference (decoder_change) and, as itself, decoder_sem; both are written by one pass into the two decoders' concat
# buffers, and the backward forms maxpool_bwd(g_pool) -/+ g_diff + g_sem inside the level's BatchNorm backward.
# ------------------------------------------------------------------------------------------------
class DualTaskLevelFn(torch.autograd.Function):
    """One encoder level of DualTaskSiameseUNet on the [t1; t2] pair batch: the difference d = a_t2 - a_t1 (B images,
    decoder_change's skip or deepest input), the semantic batch o = [a_t2; a_t1] (2B images, decoder_sem's: t2 first,
    as the reference calls decoder_sem(features_t2) first) and, below the deepest level, the next level's pooled input.
    The activation itself is never written outside those (scd_bn_relu_pool_out mode 2).  meta.extra_c / extra_s: the
    ConvT channels of the two decoders' Ups taking this level (zero-copy cat; meta.bufc / bufs the buffers)."""

    @staticmethod
    def forward(ctx, x, meta, *params):
        ctx.set_materialize_grads(False)
        meta.scope = (hip.conv_math(), hip.conv_tune())
        _, sv, y1, st1, bound = _dc_forward(x, meta.dc, 2, meta.training, meta.save, materialize=False,
                                            pool=meta.pool, x_bound=meta.x_bound)
        meta.out_bound = bound
        n2, h, w, c = y1.shape
        b = n2 // 2
        bufc = _act((b, h, w, c + meta.extra_c), y1)
        bufs = _act((n2, h, w, c + meta.extra_s), y1)
        d = bufc[..., :c] if meta.extra_c else bufc
        o = bufs[..., :c] if meta.extra_s else bufs
        sc, sh = _two_seg(st1)
        idx = nxt = None
        if not meta.last:
            nxt = _act((n2, h // 2, w // 2, c), y1)
            idx = _empty((n2, h // 2, w // 2, c), y1, dtype=torch.uint8)
        if _even(h, w):
            hip.bn_relu_pool_out(nhwc(y1), 2, sc, sh, hip.POOL_DIFF_COPY, nhwc(d), nhwc(o),
                                 nhwc(nxt) if nxt is not None else hip._NULL, idx)
        else:  # odd maps (e.g. evaluation on odd tiles): materialise, then the difference, the copies and the pooling
            a = _act(tuple(y1.shape), y1)
            hip.bn_relu_apply(nhwc(y1), 2, sc, sh, nhwc(a))
            hip.siamese_diff(nhwc(a), nhwc(d))
            hip.feature_grad(hip._NULL, None, nhwc(a[b:]), 0, nhwc(o[:b]))
            hip.feature_grad(hip._NULL, None, nhwc(a[:b]), 0, nhwc(o[b:]))
            if nxt is not None:
                hip.maxpool2_fwd(nhwc(a), nhwc(nxt), idx)
        _set_bound(d, bound)  # |a_t2 - a_t1| <= max(a_t1, a_t2) for ReLU outputs
        _set_bound(o, bound)
        meta.bufc = bufc if meta.extra_c else None
        meta.bufs = bufs if meta.extra_s else None
        if meta.save:
            ctx.meta, ctx.saved = meta, (sv, idx, b)
        return (d, o) if nxt is None else (d, o, nxt)

    @staticmethod
    def backward(ctx, g_d, g_o, g_next=None):
        meta = ctx.meta
        with hip.conv_scope(*meta.scope):
            sv, idx, b = ctx.saved
            y1 = sv[4]
            if g_o is None:  # the semantic branch took no gradient: the Siamese level's backward
                ga = _level_grad(g_next, idx, g_d, 1, y1)
            else:
                if g_d is None:
                    g_d = torch.zeros((b,) + tuple(y1.shape[1:]), device=y1.device, dtype=y1.dtype)
                ga = _PooledGrad(g_next, idx if g_next is not None else None, g_d, 2, g_o)
            gx, pg = _dc_backward(ga, sv, meta.dc, need_dx=ctx.needs_input_grad[0], pool=_bounds(y1))
        ctx.saved = None
        return (gx, None, *pg)


def run_dualtask_encoder(inc, encoder, x: torch.Tensor, training: bool, extra_c: dict, extra_s: dict):
    """Per level (level 0 first): (difference, semantic [t2; t1] batch, decoder_change buffer, decoder_sem buffer)."""
    blocks = encoder_blocks(inc, encoder)
    pool, bound = _bounds(x), None
    diffs, sems, bufc, bufs, cur = [], [], [], [], x
    try:
        for level, dc in enumerate(blocks):
            params = dc_params(dc)
            save = torch.is_grad_enabled() and (cur.requires_grad or any(p.requires_grad for p in params))
            meta = _Meta(dc=dc, training=training, save=save, last=level == len(blocks) - 1, pool=pool,
                         x_bound=bound, extra_c=extra_c.get(level, 0), extra_s=extra_s.get(level, 0))
            outs = DualTaskLevelFn.apply(cur, meta, *params)
            diffs.append(outs[0])
            sems.append(outs[1])
            bufc.append(meta.bufc)
            bufs.append(meta.bufs)
            bound = meta.out_bound
            if not meta.last:
                cur = outs[2]
    finally:
        flush_bn_counters()
    return diffs, sems, bufc, bufs


# ------------------------------------------------------------------------------------------------
# Siamese encoder with the feature difference fused in (SiameseUNet / WhateverNet streams)
# ------------------------------------------------------------------------------------------------
def _two_seg(st: _BNSaved):
    """Per-branch [2][C] coefficients (eval mode has one set for both branches)."""
    if st.nseg == 2:
        return st.scale, st.shift
    return torch.cat([st.scale, st.scale]), torch.cat([st.shift, st.shift])


class SiameseLevelFn(torch.autograd.Function):
    """One level of InConv + Encoder on the 2B-image pair batch, returning f_t2 - f_t1 (networks.py:141-150) and,
    below the deepest level, the next level's pooled input.

    The level's output activation relu(BN1(y1)) is never materialised: the difference and the next level's
    MaxPool2d read y1 through BN1 + ReLU (one pass, scd_bn_relu_pool_diff, for even maps).  The difference is written
    into channels [0, C) of the decoder's concat buffer when meta.extra names its ConvT channels (zero-copy cat,
    networks.py:449).  Backward: dL/da1 = maxpool_bwd(g_pool) -/+ g_diff (t1/t2), formed in the BatchNorm backward."""

    @staticmethod
    def forward(ctx, x, meta, *params):
        ctx.set_materialize_grads(False)
        meta.scope = (hip.conv_math(), hip.conv_tune())
        _, sv, y1, st1, bound = _dc_forward(x, meta.dc, 2, meta.training, meta.save, materialize=False,
                                            pool=meta.pool, x_bound=meta.x_bound)
        meta.out_bound = bound
        n2, h, w, c = y1.shape
        buf = _act((n2 // 2, h, w, c + meta.extra), y1)
        d = buf[..., :c] if meta.extra else buf
        sc, sh = _two_seg(st1)
        idx = nxt = None
        if not meta.last:
            nxt = _act((n2, h // 2, w // 2, c), y1)
            idx = _empty((n2, h // 2, w // 2, c), y1, dtype=torch.uint8)
        if nxt is not None and h % 2 == 0 and w % 2 == 0 and _OPTS['pool_diff']:
            hip.bn_relu_pool_diff(nhwc(y1), sc, sh, nhwc(buf, 0, c), nhwc(nxt), idx)  # one read of y1
        else:
            hip.bn_relu_siamese_diff(nhwc(y1), sc, sh, nhwc(buf, 0, c))
            if nxt is not None:
                hip.bn_relu_maxpool2_fwd(nhwc(y1), st1.nseg, st1.scale, st1.shift, nhwc(nxt), idx)
        _set_bound(d, bound)  # |a_t2 - a_t1| <= max(a_t1, a_t2) for ReLU outputs
        meta.buf = buf if meta.extra else None
        if meta.save:
            ctx.meta, ctx.saved = meta, (sv, idx)
        return (d,) if nxt is None else (d, nxt)

    @staticmethod
    def backward(ctx, g_d, g_next=None):
        meta = ctx.meta
        with hip.conv_scope(*meta.scope):
            sv, idx = ctx.saved
            ga = _level_grad(g_next, idx, g_d, 1, sv[4])
            gx, pg = _dc_backward(ga, sv, meta.dc, need_dx=ctx.needs_input_grad[0], pool=_bounds(sv[4]))
        ctx.saved = None
        return (gx, None, *pg)


def run_siamese_encoder(inc, encoder, x: torch.Tensor, training: bool, extra: dict | None = None):
    """Feature differences per level (level 0 first) and the concat buffers they live in (None where plain)."""
    blocks = encoder_blocks(inc, encoder)
    extra = extra or {}
    pool, bound = _bounds(x), None
    diffs, bufs, cur = [], [], x
    try:
        for level, dc in enumerate(blocks):
            params = dc_params(dc)
            save = torch.is_grad_enabled() and (cur.requires_grad or any(p.requires_grad for p in params))
            meta = _Meta(dc=dc, training=training, save=save, last=level == len(blocks) - 1, pool=pool,
                         x_bound=bound, extra=extra.get(level, 0))
            outs = SiameseLevelFn.apply(cur, meta, *params)
            diffs.append(outs[0])
            bufs.append(meta.buf)
            bound = meta.out_bound
            if not meta.last:
                cur = outs[1]
    finally:
        flush_bn_counters()
    return diffs, bufs


# ------------------------------------------------------------------------------------------------
# Siamese feature difference
# ------------------------------------------------------------------------------------------------
class SiameseDiffFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, feat):
        n2, h, w, c = feat.shape
        d = _act((n2 // 2, h, w, c), feat)
        hip.siamese_diff(nhwc(feat), nhwc(d))
        ctx.shape = feat.shape
        return d

    @staticmethod
    def backward(ctx, g):
        gf = _act(tuple(ctx.shape), g)
        hip.feature_grad(hip._NULL, None, nhwc(g), 1, nhwc(gf))
        return gf


def siamese_diff(feat: torch.Tensor) -> torch.Tensor:
    return SiameseDiffFn.apply(feat)


# ------------------------------------------------------------------------------------------------
# Decoder: Up x L
# ------------------------------------------------------------------------------------------------
def up_params(up) -> list:
    return [up.up.weight, up.up.bias] + dc_params(up.conv)


class DecoderFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, meta, x_deep, *rest):
        ctx.set_materialize_grads(False)
        meta.scope = (hip.conv_math(), hip.conv_tune())
        ups = meta.ups
        skips = rest[:len(ups)]
        cur = x_deep
        saved = []
        pool = _bounds(x_deep)
        head = meta.head
        for k, up in enumerate(ups):
            last_into_head = head is not None and k == len(ups) - 1
            skip = skips[k]
            b, h, w, cs = skip.shape
            _, hc, wc, cu = cur.shape
            convT = up.up
            cto = convT.out_channels
            pad_y, pad_x = h - 2 * hc, w - 2 * wc  # networks.py:437-443 (diffY, diffX)
            if pad_y < 0 or pad_x < 0:
                raise ValueError(f"Up: upsampled map {2 * hc}x{2 * wc} is larger than the skip {h}x{w}")
            buf = meta.cat_buffers[k] if meta.cat_buffers is not None else None
            if (buf is not None and buf.data_ptr() == skip.data_ptr() and tuple(buf.shape) == (b, h, w, cs + cto)
                    and skip.stride(2) == cs + cto):
                cat = buf  # the encoder wrote the skip into channels [0, cs) already (zero-copy cat)
            else:
                cat = _act((b, h, w, cs + cto), skip)
                hip.feature_grad(hip._NULL, None, nhwc(skip), 0, nhwc(cat, 0, cs))  # skip -> cat[..., :cs]
            wT = packed_convT2x2(convT.weight, 0)
            # h2: the concat's own bound, seeded with the skip's and raised by the ConvT epilogue to max |up| (F.pad's
            # zero border adds nothing); the skip's bound, also read by the encoder's weight grads, stays as it is.
            # The ConvT reads cur through cur's bound.
            cur_bound = _bound_of(cur, pool)
            cat_bound = skip_bound = None
            if pool is not None:
                cat_bound, skip_bound = pool.take(), _bound_of(skip, pool)
            # the ConvT epilogue raises a bound on the split kernels only (src.c % 16 == 0), seeded with the skip's
            # inside the launch (dst_bound_seed); else a copy of the skip's bound and one absmax pass
            epi_bound = cat_bound if hip.conv_math() != 'f32' and cu % 16 == 0 else None
            seed = skip_bound if epi_bound is not None else None
            if cat_bound is not None and epi_bound is None:
                cat_bound.copy_(skip_bound)
            if pad_y or pad_x:
                # ConvT into its own map, then F.pad's zero border and placement in one window copy
                upm = _act((b, 2 * hc, 2 * wc, cto), skip)
                hip.conv_igemm(nhwc(cur), hc, wc, 1, TAPS_1, wT, 4 * cto, convT.bias, nhwc(upm), store_mode=1,
                               src_bound=cur_bound, dst_bound=epi_bound, dst_bound_seed=seed)
                hip.window_copy(nhwc(upm), nhwc(cat, cs, cto), -(pad_y // 2), -(pad_x // 2))
            else:
                hip.conv_igemm(nhwc(cur), hc, wc, 1, TAPS_1, wT, 4 * cto, convT.bias, nhwc(cat, cs, cto),
                               store_mode=1, src_bound=cur_bound, dst_bound=epi_bound, dst_bound_seed=seed)
            if cat_bound is not None and epi_bound is None:
                hip.absmax_bound(nhwc(cat, cs, cto), cat_bound)
            last_raw = meta.raw and k == len(ups) - 1
            a, sv, y1, st1, _ = _dc_forward(cat, up.conv, meta.nseg, meta.training, meta.save,
                                            materialize=not (last_into_head or last_raw), pool=pool, x_bound=cat_bound)
            saved.append((cur, cat, cs, sv, cur_bound))
            cur = a
            if last_raw:
                # the decoder's last conv output y1 itself: its BatchNorm + ReLU are read by the heads (HeadsFn), which
                # also run that BatchNorm's backward; meta.raw_state carries the coefficients to them
                cur = y1
                meta.raw_state = (st1, up.conv)
            if last_into_head:
                # OutConv (networks.py:457) reading relu(BN1(y1)) through the coefficients: the decoder's output
                # activation is never written
                n, h, w, c = y1.shape
                hw_, hb_ = rest[-2], rest[-1]
                n_out = hw_.shape[0]
                w2 = hw_.detach().reshape(n_out, c).contiguous()
                cur = _empty((n, n_out, h, w), y1)
                hip.conv1x1_fwd_bn(nhwc(y1), st1.scale, st1.shift, st1.nseg, w2, hb_, n_out, cur)
                ctx.head = (y1, st1, w2, n_out, hw_.shape, hb_ is not None)
        if meta.save:
            ctx.meta = meta
            ctx.saved = saved
        return cur

    @staticmethod
    def backward(ctx, g_out):
        with hip.conv_scope(*ctx.meta.scope):
            return DecoderFn._backward(ctx, g_out)

    @staticmethod
    def _backward(ctx, g_out):
        meta, saved = ctx.meta, ctx.saved
        ups = meta.ups
        n = len(ups)
        g_skips = [None] * n
        grads = [None] * (10 * n)
        head_grads = [None, None] if meta.head is not None else []
        g = g_out
        if g is None:
            return (None, None, *g_skips, *grads, *head_grads)
        if meta.head is None:
            g = g.contiguous()  # e.g. the gradient of a permuted (NCHW) view of the output, from a standalone Up
        pool = _bounds(g)
        if meta.head is not None:
            y1, st1, w2, n_out, wshape, has_bias = ctx.head
            g = g.contiguous()
            gw = _empty(tuple(wshape), y1)
            gb = _empty((n_out,), y1) if has_bias else None
            ws = _ws(hip.conv1x1_workspace_bytes(nhwc(y1), n_out), y1)
            # the head's weight grad comes from its BatchNorm's backward pass over y1 (scd_bn_relu_backward_head
            # w_grad); here only its bias grad
            fold = _OPTS['head_wgrad_in_bn_bwd']
            hip.conv1x1_bwd_bn(nhwc(y1), st1.scale, st1.shift, st1.nseg, w2, g, n_out, None if fold else gw, gb, ws)
            head_grads = [gw, gb]
            g = _HeadGrad(g, w2, n_out, gw if fold else None)
            ctx.head = None
        for k in range(n - 1, -1, -1):
            up = ups[k]
            cur, cat, cs, sv, cur_bound = saved[k]
            g_cat, pg = _dc_backward(g, sv, up.conv, need_dx=True, pool=pool, dy1_given=meta.raw and k == n - 1)
            g_skips[k] = g_cat[..., :cs]
            convT = up.up
            cto = convT.out_channels
            b, hc, wc, cu = cur.shape
            bb, hh, ww, _ = g_cat.shape
            if (hh, ww) != (2 * hc, 2 * wc):  # backward of F.pad: crop the ConvT's window out of g_cat
                g_up_t = _act((b, 2 * hc, 2 * wc, cto), g_cat)
                hip.window_copy(nhwc(g_cat, cs, cto), nhwc(g_up_t), (hh - 2 * hc) // 2, (ww - 2 * wc) // 2)
                g_up = nhwc(g_up_t)
                hh, ww = 2 * hc, 2 * wc
            else:
                g_up = nhwc(g_cat, cs, cto)
            # ConvT data grad: 4-tap stride-2 gather of g_cat's up half (h2: through g_cat's bound, raised by the
            # DoubleConv data grad that wrote it)
            g_cur = torch.empty_like(cur)
            gcat_bound = _bound_of(g_cat, pool)
            # h2: the kernel raises g_cur's bound as it stores (a BatchNorm backward formed inside the next weight
            # grad scales its dy by a bound derived from it, _bn_backward_in_wgrad)
            wT = packed_convT2x2(convT.weight, 1)
            gcur_bound = None
            if pool is not None and _OPTS['bn_bwd_in_wgrad'] and k > 0 and \
                    hip.igemm_arith(g_up, hc, wc, 2, TAPS_2X2, wT, cu, nhwc(g_cur), src_bound=gcat_bound) == 'h2':
                gcur_bound = pool.take()
            hip.conv_igemm(g_up, hc, wc, 2, TAPS_2X2, wT, cu, None, nhwc(g_cur), src_bound=gcat_bound,
                           dst_bound=gcur_bound)
            _set_bound(g_cur, gcur_bound)
            # ConvT weight grad: rows = convT input, src = g_up gathered with stride 2 (h2: both bounds)
            # (and its bias grad: the kernel sums the g_up columns it stages, scd_wgrad_t.src_colsum)
            d, nsplit, nbytes = hip.wgrad_plan(nhwc(cur), g_up, 2, TAPS_2X2, None, cur_bound, gcat_bound)
            slabs = _empty((nbytes // 4,), cur)
            colsum = None
            if _OPTS['convT_bias_in_wgrad'] and hip.wgrad_colsum_supported(d):
                colsum = _empty((nsplit * 4 * cto,), cur)
                d.src_colsum = colsum.data_ptr()
            hip.conv_wgrad(d, slabs)
            gwT = torch.empty_like(convT.weight)
            hip.wgrad_finalize(slabs, nsplit, cu, 4, cto, 1, cto, gwT)
            gbT = _empty((cto,), cur)
            if colsum is not None:
                hip.wgrad_colsum_finalize(colsum, nsplit, 4, cto, gbT)
            else:
                hip.channel_sum(g_up, gbT, _ws(hip.bn_workspace_bytes(bb, hh, ww, cto, 1), cur))
            grads[10 * k:10 * k + 10] = [gwT, gbT] + pg
            g = g_cur
        ctx.saved = None
        return (None, g, *g_skips, *grads, *head_grads)


def decoder_cat_channels(decoder, n_levels: int) -> dict:
    """{encoder level: ConvT output channels of the Up that takes that level's skip}: the concat buffer extent
    an encoder level can write its skip into (run_siamese_encoder `extra`)."""
    ups = list(decoder.up_seq.values())
    return {n_levels - 2 - k: up.up.out_channels for k, up in enumerate(ups)}


def run_decoder(decoder, features: list, training: bool, cat_buffers: list | None = None, head=None, nseg: int = 1):
    """`features` in the reference's order: [deepest, ..., level 0] (Encoder.forward's reversed list).
    `cat_buffers`: per Up (same order as decoder.up_seq), the concat buffer its skip already lives in, or None.
    `head` (an OutConv that is the decoder output's only reader): returns the head's logits (NCHW) instead, with
    the head reading the last BatchNorm + ReLU through its coefficients (scd_conv1x1_fwd_bn) and its backward
    feeding that BatchNorm's backward directly (scd_bn_relu_backward_head); results are bit-identical to
    run_head(head, run_decoder(...)).  head='raw': returns a RawDecoderOut for run_heads (several heads, or a head over
    two decoders).  nseg: BatchNorm segments of the batch (decoder_sem's [t2; t1] batch: 2)."""
    return run_ups(list(decoder.up_seq.values()), features, training, cat_buffers, head, nseg)


@dataclass
class RawDecoderOut:
    """A decoder's output left unmaterialised for run_heads: its last conv output y (NHWC, the autograd output of the
    decoder stage), the BatchNorm coefficients / statistics the heads read it through, and that DoubleConv."""
    y: torch.Tensor
    st: '_BNSaved'
    dc: object


def run_ups(ups: list, features: list, training: bool, cat_buffers: list | None = None, head=None, nseg: int = 1):
    """Up blocks in sequence (Decoder.forward, networks.py:375-382): features[0] is the deepest map, features[1 + k]
    the skip of ups[k]."""
    raw = isinstance(head, str) and head == 'raw'
    if raw:
        head = None
    if head is not None and (not _OPTS['fuse_head'] or head.conv.out_channels > 4):
        return run_head(head, run_ups(ups, features, training, cat_buffers, nseg=nseg))
    params = [p for up in ups for p in up_params(up)]
    if head is not None:
        params += [head.conv.weight, head.conv.bias]
        if head.conv.bias is None:
            raise ValueError("run_decoder: the fused head expects OutConv's bias (networks.py:457)")
    save = torch.is_grad_enabled() and (any(p.requires_grad for p in params) or any(f.requires_grad for f in features))
    meta = _Meta(ups=ups, training=training, save=save, cat_buffers=cat_buffers, head=head, raw=raw, nseg=nseg,
                 raw_state=None)
    try:
        out = DecoderFn.apply(meta, features[0], *features[1:1 + len(ups)], *params)
    finally:
        flush_bn_counters()
    if raw:
        st, dc = meta.raw_state
        return RawDecoderOut(out, st, dc)
    return out


class HeadsFn(torch.autograd.Function):
    """OutConv heads (networks.py:454-461) over one or two decoder outputs, each read through its last BatchNorm + ReLU
    (networks.py:380-381): DualStreamUNet's outc over cat(x_stream1, x_stream2) (networks.py:117-120) and WhateverNet /
    WhateverNet2's outc_stream1, outc_stream2 and outc_fusion (networks.py:241-263, 288-310) in ONE launch
    (scd_conv1x1_fwd_bn2): each decoder output is read once for all heads, and neither it nor the cat is written.
    Output: [n, K, h, w], the heads' logits stacked along channels (K = their output channels, <= 4).
    Backward: per source, that BatchNorm's backward with dL/da = sum_k g_k w_k[source] formed on the fly and the heads'
    weight grads from the same pass (scd_bn_relu_backward_head over the stacked [K][C_s] weights); it returns dL/dy
    of the source to its decoder stage (DecoderFn raw mode) plus the BatchNorm's and conv bias's gradients."""

    @staticmethod
    def forward(ctx, meta, *args):
        meta.scope = (hip.conv_math(), hip.conv_tune())  # the backward's bounds follow the model's arithmetic
        srcs, heads = meta.srcs, meta.heads
        ns = len(srcs)
        ys = args[:ns]
        hp = args[4 * ns:]
        y0 = ys[0]
        n, h, w, _ = y0.shape
        cs = [y.shape[3] for y in ys]
        offs = [sum(cs[:i]) for i in range(ns)]
        ctot = sum(cs)
        K = sum(hp[2 * j].shape[0] for j in range(len(heads)))
        wall = torch.zeros((K, ctot), device=y0.device, dtype=_F32)
        ball = torch.zeros((K,), device=y0.device, dtype=_F32)
        rows, k0 = [], 0
        with torch.no_grad():
            for j, sel in enumerate(heads):
                wt, bt = hp[2 * j], hp[2 * j + 1]
                no = wt.shape[0]
                w2 = wt.detach().reshape(no, -1)
                col = 0
                for si in sel:  # the head's input channels: its sources concatenated in the listed order
                    wall[k0:k0 + no, offs[si]:offs[si] + cs[si]] = w2[:, col:col + cs[si]]
                    col += cs[si]
                if col != w2.shape[1]:
                    raise ValueError(f"head {j}: weight takes {w2.shape[1]} channels, its sources give {col}")
                if bt is not None:
                    ball[k0:k0 + no] = bt.detach()
                rows.append((k0, no, tuple(sel), tuple(wt.shape), bt is not None))
                k0 += no
        out = _empty((n, K, h, w), y0)
        sa, sb = srcs[0].st, srcs[1].st if ns > 1 else None
        hip.conv1x1_fwd_bn2(nhwc(ys[0]), sa.scale, sa.shift, nhwc(ys[1]) if ns > 1 else hip._NULL,
                            sb.scale if sb else None, sb.shift if sb else None, sa.nseg, wall, ball, K, out)
        ctx.meta = meta
        ctx.state = (ys, wall, rows, offs, cs, K)
        return out

    @staticmethod
    def backward(ctx, g):
        with hip.conv_scope(*ctx.meta.scope):
            return HeadsFn._backward(ctx, g)

    @staticmethod
    def _backward(ctx, g):
        meta = ctx.meta
        ys, wall, rows, offs, cs, K = ctx.state
        ctx.state = None
        ns = len(meta.srcs)
        if g is None:
            return (None,) * (1 + 4 * ns + 2 * len(rows))
        g = g.contiguous()
        pool = _bounds(ys[0])
        dys, bn_grads, wgs = [], [], []
        for i, (y, src) in enumerate(zip(ys, meta.srcs)):
            st, dc = src.st, src.dc
            if st.smean is None:
                raise RuntimeError("backward through an eval-mode BatchNorm is not supported (call net.train())")
            bn, conv = dc.conv[4], dc.conv[3]
            n, h, w, c = y.shape
            ws_ = wall[:, offs[i]:offs[i] + cs[i]].contiguous()
            dy = torch.empty_like(y)
            dgamma, dbeta = _empty((c,), y), _empty((c,), y)
            dbias = _empty((c,), y) if conv.bias is not None else None
            wg = _empty((K, c), y)
            db = _take(pool)
            ws = _ws(hip.bn_head_workspace_bytes(n, h, w, c, st.nseg, K), y)
            hip.bn_relu_backward_head(nhwc(y), g, ws_, K, st.nseg, st.smean, st.sinv, bn.weight, st.scale, st.shift,
                                      dgamma, dbeta, dbias, nhwc(dy), ws, db, wg)
            dys.append(_set_bound(dy, db))
            bn_grads += [dgamma, dbeta, dbias]
            wgs.append(wg)
        y0, st0 = ys[0], meta.srcs[0].st
        gb = _empty((K,), y0)
        ws = _ws(hip.conv1x1_workspace_bytes(nhwc(y0), K), y0)
        hip.conv1x1_bwd_bn(nhwc(y0), st0.scale, st0.shift, st0.nseg, wall[:, :cs[0]].contiguous(), g, K, None, gb, ws)
        head_grads = []
        for k0, no, sel, wshape, has_b in rows:
            gw = torch.cat([wgs[si][k0:k0 + no] for si in sel], dim=1).reshape(wshape)
            head_grads += [gw, gb[k0:k0 + no].clone() if has_b else None]
        return (None, *dys, *bn_grads, *head_grads)


def run_heads(sources: list, heads: list) -> list:
    """heads: [(OutConv, (source indices in its input's channel order))] over `sources` (RawDecoderOut of run_decoder
    head='raw'); returns each head's NCHW logits (channel slices of one stacked output).  Takes <= 2 sources of one
    (n, h, w) and BatchNorm segment count and <= 4 output channels over all heads, each with its bias (OutConv's)."""
    y0 = sources[0].y
    if not 1 <= len(sources) <= 2 or any(s.y.shape[:3] != y0.shape[:3] or s.st.nseg != sources[0].st.nseg
                                         or s.y.shape[3] % 4 for s in sources):
        raise ValueError("run_heads: 1-2 decoder outputs of one (n, h, w) and segment count, channels in multiples of 4")
    if sum(o.conv.out_channels for o, _ in heads) > 4 or any(o.conv.bias is None for o, _ in heads):
        raise ValueError("run_heads: at most 4 output channels over all heads, each head with a bias")
    params = [p for s in sources for p in (s.dc.conv[4].weight, s.dc.conv[4].bias, s.dc.conv[3].bias)]
    for outc, _ in heads:
        params += [outc.conv.weight, outc.conv.bias]
    meta = _Meta(srcs=sources, heads=[tuple(sel) for _, sel in heads])
    out = HeadsFn.apply(meta, *[s.y for s in sources], *params)
    res, k0 = [], 0
    for outc, _ in heads:
        no = outc.conv.out_channels
        res.append(out[:, k0:k0 + no])
        k0 += no
    return res


# ------------------------------------------------------------------------------------------------
# OutConv 1x1 head
# ------------------------------------------------------------------------------------------------
class HeadFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias):
        n, h, w, c = x.shape
        n_out = weight.shape[0]
        out = _empty((n, n_out, h, w), x)
        w2 = weight.detach().reshape(n_out, c).contiguous()
        hip.conv1x1_fwd(nhwc(x), w2, bias, n_out, out)
        ctx.save_for_backward(x, w2)
        ctx.n_out = n_out
        ctx.wshape = weight.shape
        ctx.has_bias = bias is not None
        return out

    @staticmethod
    def backward(ctx, g):
        x, w2 = ctx.saved_tensors
        n_out = ctx.n_out
        gx = torch.empty_like(x)
        gw = _empty(tuple(ctx.wshape), x)
        gb = _empty((n_out,), x) if ctx.has_bias else None
        ws = _ws(hip.conv1x1_workspace_bytes(nhwc(x), n_out), x)
        hip.conv1x1_bwd(nhwc(x), w2, g.contiguous(), n_out, nhwc(gx), False, gw, gb, ws)
        return gx, gw, gb


def run_head(outc, x: torch.Tensor) -> torch.Tensor:
    """OutConv (networks.py:454-461) of an NHWC activation -> NCHW logits.  The 1x1 kernel takes up to 4 output
    channels per launch and channel counts in multiples of 4: wider heads run in groups of 4 outputs, and a source
    whose channels are not a multiple of 4 is zero-padded with its weight (both differentiable: the padding's
    gradient is dropped)."""
    w, b = outc.conv.weight, outc.conv.bias
    c = x.shape[3]
    if c % 4:
        cp = (c + 3) // 4 * 4
        x = torch.nn.functional.pad(x, (0, cp - c))
        w = torch.nn.functional.pad(w, (0, 0, 0, 0, 0, cp - c))
    n_out = w.shape[0]
    if n_out <= 4:
        return HeadFn.apply(x, w, b)
    outs = [HeadFn.apply(x, w[i:i + 4], None if b is None else b[i:i + 4]) for i in range(0, n_out, 4)]
    return torch.cat(outs, dim=1)


# ------------------------------------------------------------------------------------------------
# Standalone building blocks (DoubleConv / InConv / Down, networks.py:386-426) for callers that use a block on its
# own (e.g. assessment_semantics.py:34 calls net.outc_sem_change directly).  The model forwards do not come here:
# they run whole stages (EncoderLevelFn, SiameseLevelFn, DecoderFn).
# ------------------------------------------------------------------------------------------------
def to_nhwc(x: torch.Tensor, c_pad: int | None = None) -> torch.Tensor:
    """NCHW -> contiguous NHWC fp32 (zero channels up to c_pad), differentiable."""
    hip.ensure_device(x)
    if x.dim() != 4:
        raise ValueError(f"expected a (B, C, H, W) tensor, got {tuple(x.shape)}")
    y = x.float().permute(0, 2, 3, 1)
    if c_pad is not None and c_pad > y.shape[3]:
        y = torch.nn.functional.pad(y, (0, c_pad - y.shape[3]))
    return y.contiguous()


def to_nchw(y: torch.Tensor) -> torch.Tensor:
    return y.permute(0, 3, 1, 2).contiguous()


class BlockFn(torch.autograd.Function):
    """One DoubleConv on an NHWC batch (one BatchNorm segment), optionally behind MaxPool2d(2) (Down)."""

    @staticmethod
    def forward(ctx, x, meta, *params):
        ctx.set_materialize_grads(False)
        meta.scope = (hip.conv_math(), hip.conv_tune())
        pool = _bounds(x)
        cur, idx = x, None
        if meta.maxpool:
            n, h, w, c = x.shape
            cur = _act((n, h // 2, w // 2, c), x)
            idx = _empty((n, h // 2, w // 2, c), x, dtype=torch.uint8)
            hip.maxpool2_fwd(nhwc(x), nhwc(cur), idx)
        a, sv, _, _, _ = _dc_forward(cur, meta.dc, 1, meta.training, meta.save, pool=pool)
        if meta.save:
            ctx.meta, ctx.saved = meta, (idx, sv, tuple(x.shape))
        return a

    @staticmethod
    def backward(ctx, g):
        if g is None:
            return (None, None) + (None,) * 8
        meta = ctx.meta
        with hip.conv_scope(*meta.scope):
            idx, sv, xshape = ctx.saved
            need_dx = ctx.needs_input_grad[0]
            gx, pg = _dc_backward(g.contiguous(), sv, meta.dc, need_dx=need_dx, pool=_bounds(g))
            if need_dx and meta.maxpool:  # MaxPool2d backward through the argmax bytes
                gfull = _act(xshape, g)
                hip.feature_grad(nhwc(gx), idx, hip._NULL, 0, nhwc(gfull))
                gx = gfull
        ctx.saved = None
        return (gx, None, *pg)


def run_block(dc, x: torch.Tensor, training: bool, maxpool: bool = False) -> torch.Tensor:
    """DoubleConv `dc` (networks.py:386-402) of an NHWC batch, after MaxPool2d(2) when `maxpool` (Down,
    networks.py:415-426); NHWC out."""
    params = dc_params(dc)
    save = torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in params))
    meta = _Meta(dc=dc, training=training, save=save, maxpool=maxpool)
    try:
        return BlockFn.apply(x, meta, *params)
    finally:
        flush_bn_counters()


# ------------------------------------------------------------------------------------------------
# Channel concatenation of NHWC stage outputs (fusion heads)
# ------------------------------------------------------------------------------------------------
class CatFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, *xs):
        n, h, w, _ = xs[0].shape
        cs = [x.shape[3] for x in xs]
        out = _act((n, h, w, sum(cs)), xs[0])
        off = 0
        for x, c in zip(xs, cs):
            hip.feature_grad(hip._NULL, None, nhwc(x), 0, nhwc(out, off, c))
            off += c
        ctx.cs = cs
        return out

    @staticmethod
    def backward(ctx, g):
        outs, off = [], 0
        for c in ctx.cs:
            outs.append(g[..., off:off + c])
            off += c
        return tuple(outs)


def cat_channels(*xs) -> torch.Tensor:
    return CatFn.apply(*xs)


# ------------------------------------------------------------------------------------------------
# power_jaccard_loss
# ------------------------------------------------------------------------------------------------
# Exact-DataParallel loss (parallel.wrap_ddp(exact_dataparallel=True)): a callable that SUM-all-reduces a device
# tensor in place across the ranks, applied to the loss kernels' partial sums, so every rank forms ONE loss over the
# batch of all ranks, as nn.DataParallel's gathered-batch loss does (utils/networks.py:27, train_supervised.py:75).
# It is scoped, not process-wide: only a loss formed inside `loss_reduction(fn)` (trainers.step_loss enters it for a
# model wrapped in that mode, parallel.loss_scope) runs the collective; any other loss in the process (a rank-0
# validation loss, a second model) stays local and issues no collective.
_LOSS_ALLREDUCE = contextvars.ContextVar('scd_loss_allreduce', default=None)


@contextlib.contextmanager
def loss_reduction(fn):
    """Inside: the loss kernels' partial sums are reduced by fn (None: local)."""
    tok = _LOSS_ALLREDUCE.set(fn)
    try:
        yield
    finally:
        _LOSS_ALLREDUCE.reset(tok)


def current_loss_reduction():
    return _LOSS_ALLREDUCE.get()


class PJaccardFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target):
        logits = logits.contiguous().float()
        target = target.contiguous().float()
        if logits.numel() != target.numel():
            raise ValueError(f"power_jaccard_loss: {logits.numel()} logits vs {target.numel()} targets")
        sums = _empty((3,), logits)
        loss = _empty((), logits)
        ws = _ws(hip.pjaccard_workspace_bytes(logits.numel()), logits)
        hip.pjaccard_fwd(logits, target, sums, loss, ws)
        red = _LOSS_ALLREDUCE.get()
        if red is not None:  # global {I, sum(p^2 + t^2)}, then D and the loss re-formed from them
            red(sums)
            hip.pjaccard_loss_from_sums(sums, loss)
        ctx.save_for_backward(logits, target, sums)
        return loss

    @staticmethod
    def backward(ctx, g):
        logits, target, sums = ctx.saved_tensors
        gl = torch.empty_like(logits)
        gt = torch.empty_like(target) if ctx.needs_input_grad[1] else None
        hip.pjaccard_bwd(logits, target, sums, g.contiguous(), gl, gt)
        return gl, gt


def power_jaccard(logits: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    hip.ensure_device(logits)
    return PJaccardFn.apply(logits, target)


# ------------------------------------------------------------------------------------------------
# Fused multi-term power-Jaccard (dual-task and MMCR trainers)
# ------------------------------------------------------------------------------------------------
class MultiJaccardFn(torch.autograd.Function):
    """sum_t coef_t * [|sel_t| > 0] * power_jaccard_loss(logits_t[sel_t], target_t[sel_t]) in one fused pass
    (scd_jaccard_multi_fwd/bwd).  spec: per term (logits index, target index, coef, select, soft) into `tensors`;
    select 0 = all samples, 1 = labelled, 2 = unlabelled; a soft target is the logits of sigmoid targets and gets a
    gradient.  No host sync: empty subsets are dropped on the device."""

    @staticmethod
    def forward(ctx, spec, labeled, *tensors):
        ts = [t.contiguous().float() for t in tensors]
        n_samples = ts[0].shape[0]
        pixels = ts[0].numel() // n_samples
        for t in ts:
            if t.numel() != n_samples * pixels:
                raise ValueError(f"multi-term Jaccard: tensor of {t.numel()} elements, expected {n_samples * pixels}")
        lab = labeled.to(device=ts[0].device, dtype=torch.uint8).contiguous()
        terms = [dict(logits=ts[li], target=ts[ti], coef=c, select=sel, soft=soft) for li, ti, c, sel, soft in spec]
        sums = _empty((len(spec), 4), ts[0])
        loss = _empty((), ts[0])
        hip.jaccard_multi_fwd(terms, lab, n_samples, pixels, sums, loss)
        red = _LOSS_ALLREDUCE.get()
        if red is not None:  # exact-DataParallel: every term over the samples of all ranks
            red(sums)
            hip.jaccard_multi_loss_from_sums(terms, sums, loss)
        ctx.spec, ctx.dims = spec, (n_samples, pixels)
        ctx.save_for_backward(lab, sums, *ts)
        return loss

    @staticmethod
    def backward(ctx, g):
        lab, sums, *ts = ctx.saved_tensors
        n_samples, pixels = ctx.dims
        need = ctx.needs_input_grad[2:]
        grads = [torch.empty_like(t) if need[i] else None for i, t in enumerate(ts)]
        # the sample sets each gradient is written on; they must not overlap (a tensor in two terms over the same
        # samples would need its gradients summed), and a single partial writer zero-fills the rest
        writers = [[] for _ in ts]
        for k, (li, ti, _, sel, soft) in enumerate(ctx.spec):
            writers[li].append((k, 1, sel))
            if soft:
                writers[ti].append((k, 2, sel))
        zero = [0] * len(ctx.spec)
        for i, w in enumerate(writers):
            sels = [sel for _, _, sel in w]
            if len(sels) > 1 and (0 in sels or len(set(sels)) != len(sels)):
                raise NotImplementedError("multi-term Jaccard: a tensor in two terms over overlapping samples")
            if grads[i] is not None and len(w) == 1 and sels[0] != 0:
                zero[w[0][0]] |= w[0][1]
        terms = [dict(logits=ts[li], target=ts[ti], coef=c, select=sel, soft=soft, glogits=grads[li],
                      gtarget=grads[ti] if soft else None, zero=zero[k])
                 for k, (li, ti, c, sel, soft) in enumerate(ctx.spec)]
        hip.jaccard_multi_bwd(terms, lab, n_samples, pixels, sums, g.contiguous())
        return (None, None, *grads)


def multi_jaccard(spec, labeled: torch.Tensor, *tensors) -> torch.Tensor:
    hip.ensure_device(tensors[0])
    return MultiJaccardFn.apply(spec, labeled, *tensors)
