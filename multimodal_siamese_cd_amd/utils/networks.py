"""Drop-in replacement for the reference's `utils.networks` (utils/networks.py), MI355X-native.

Same public surface as the reference: `create_network(cfg)` (networks.py:12-27), `save_checkpoint`
(30-38), `load_checkpoint` (41-56) and the model classes UNet (59-79), DualStreamUNet (82-120),
SiameseUNet (123-154), DualTaskSiameseUNet (157-197), WhateverNet (200-263), WhateverNet2 (266-310),
Encoder (313-343), Decoder (346-382), DoubleConv (386-402), InConv (405-412), Down (415-426),
Up (429-451), OutConv (454-461).  Constructor arguments, submodule attribute paths, parameter shapes
(OIHW) and default initialisation are identical, so `state_dict()` keys and checkpoints interchange
(e.g. `module.inc.conv.conv.0.weight`).

What differs is the execution: the model-level forward runs every stage through the HIP kernels of
libscd (via multimodal_siamese_cd_amd.engine) on NHWC fp32 buffers, with the Siamese encoder run as one
2B-image batch whose BatchNorm statistics are segmented per branch.  The building blocks (Encoder, Decoder,
DoubleConv, InConv, Down, Up, OutConv) are callable on their own as in the reference (NCHW in, NCHW out, autograd),
on the same kernels; the model forwards do not call them but run whole stages.

Every model carries the conv arithmetic its config asks for (`conv_math`, engine.conv_math_for: MODEL.CONV_MATH,
else MODEL.PRECISION 'fp32' -> h2, 'bf16' -> bf16) and runs its forward and backward in that arithmetic
(hip.conv_scope), so models of different precision coexist in one process.
"""
from __future__ import annotations

from collections import OrderedDict
from pathlib import Path

import torch
import torch.nn as nn

from .. import engine, hip


def _pad8(c: int) -> int:
    return (c + 7) // 8 * 8


def _padded_topology(cfg):
    """The channel counts the kernels run a TOPOLOGY at (multiples of 8, the MFMA K granule), or None when it needs
    no padding."""
    topo = [int(t) for t in cfg.MODEL.TOPOLOGY]
    if any(t < 1 for t in topo):
        raise ValueError(f"MODEL.TOPOLOGY entries must be positive, got {topo}")
    return [_pad8(t) for t in topo] if any(t % 8 for t in topo) else None


def _dim_map(real: int, padded: int, device, halves: bool = False):
    """Positions of a parameter dimension's real channels in the padded twin's: a prefix, or (`halves`: the concat
    inputs -- Up's DoubleConv after cat([skip, up]), the fusion heads after the cat of two decoders) two halves, each
    padded on its own."""
    if padded == real:
        return None
    if halves:
        h = real // 2
        if real % 2 or padded != 2 * _pad8(h):
            raise ValueError(f"no two-half channel layout maps {real} onto {padded}")
        return torch.cat([torch.arange(h, device=device), torch.arange(h, device=device) + padded // 2])
    if padded != _pad8(real):
        raise ValueError(f"no channel layout maps {real} onto {padded}")
    return torch.arange(real, device=device)


def _concat_input(model_type: str, name: str) -> bool:
    """Parameters whose input dimension is a concat of two equally wide feature maps (networks.py:449, 119, 258)."""
    if '.up_seq.' in name and name.endswith('.conv.conv.0.weight'):
        return True
    return (model_type == 'dualstreamunet' and name == 'outc.conv.weight') or name == 'outc_fusion.conv.weight'


def _scatter(t: torch.Tensor, shape, maps) -> torch.Tensor:
    """t placed into zeros of `shape` at the per-dimension positions `maps` (differentiable in t)."""
    for d, m in enumerate(maps):
        if m is not None:
            sz = list(t.shape)
            sz[d] = shape[d]
            t = t.new_zeros(sz).index_copy(d, m, t)
    return t


def _gather(t: torch.Tensor, maps) -> torch.Tensor:
    for d, m in enumerate(maps):
        if m is not None:
            t = t.index_select(d, m)
    return t


class ModelWrapper(nn.Module):
    """Single-process stand-in for the reference's `nn.DataParallel(model)` (networks.py:27).

    On one device DataParallel is a pass-through (torch/nn/parallel/data_parallel.py:146-149); this
    wrapper keeps its observable contract — `.module` and the `module.` state_dict prefix.  Multi-GPU
    training uses one process per GPU (multimodal_siamese_cd_amd.parallel.wrap_ddp) instead.
    """

    def __init__(self, module: nn.Module):
        super().__init__()
        self.module = module

    def forward(self, *args, **kwargs):
        return self.module(*args, **kwargs)


def create_network(cfg):
    t = cfg.MODEL.TYPE
    if t == 'unet':
        model = UNet(cfg)
    elif t == 'dualstreamunet':
        model = DualStreamUNet(cfg)
    elif t == 'siameseunet':
        model = SiameseUNet(cfg)
    elif t == 'dtsiameseunet':
        model = DualTaskSiameseUNet(cfg)
    elif t == 'whatevernet':
        model = WhateverNet(cfg)
    elif t == 'whatevernet2':
        model = WhateverNet2(cfg)
    else:
        raise Exception(f'Unknown network ({t}).')
    engine.register_weight_group(model)  # per-step batched weight packing (engine.packed_conv3x3)
    return ModelWrapper(model)


def save_checkpoint(network, optimizer, epoch, step, cfg):
    save_file = Path(cfg.PATHS.OUTPUT) / 'networks' / f'{cfg.NAME}_checkpoint{epoch}.pt'
    save_file.parent.mkdir(exist_ok=True)
    torch.save({'step': step, 'network': network.state_dict(), 'optimizer': optimizer.state_dict()}, save_file)


def load_checkpoint(epoch, cfg, device, net_file: Path = None):
    net = create_network(cfg)
    net.to(device)
    save_file = net_file if net_file is not None else Path(cfg.PATHS.OUTPUT) / 'networks' / f'{cfg.NAME}_checkpoint{epoch}.pt'
    checkpoint = torch.load(save_file, map_location=device, weights_only=True)
    optimizer = torch.optim.AdamW(net.parameters(), lr=cfg.TRAINER.LR, weight_decay=0.01)
    net.load_state_dict(checkpoint['network'])
    optimizer.load_state_dict(checkpoint['optimizer'])
    return net, optimizer, checkpoint['step']


def _band_counts(cfg):
    return len(cfg.DATALOADER.S1_BANDS), len(cfg.DATALOADER.S2_BANDS)


class _HipNet(nn.Module):
    """The part every model family shares: topology check, config, arithmetic; forward runs in the model's
    arithmetic (a block called on its own runs in the caller's, hip.conv_scope / the process default)."""

    def __init__(self, cfg):
        super().__init__()
        self.cfg = cfg
        self.conv_math = engine.conv_math_for(cfg)
        # activations / gradients in HBM: bf16 for the bf16 configs (engine.act_storage_for), fp32 otherwise
        self.act_storage = engine.act_storage_for(cfg, self.conv_math)
        object.__setattr__(self, '_twin_topo', _padded_topology(cfg))
        object.__setattr__(self, '_twin', None)

    def forward(self, x_t1, x_t2):
        # levels: the input map and one per Down (Encoder: len(TOPOLOGY) of them)
        st = engine.storage_for_input(self.act_storage, x_t1.shape[-2], x_t1.shape[-1],
                                      len(self.cfg.MODEL.TOPOLOGY) + 1)
        with hip.conv_scope(self.conv_math), engine.storage_scope(st):
            if self._twin_topo is not None:
                return self._twin_forward(x_t1, x_t2)
            return self._forward(x_t1, x_t2)

    # Channel counts off the kernels' granule (any reference TOPOLOGY, e.g. [12, 20]).  The model keeps the reference's
    # parameter shapes (state_dict, checkpoints, optimizer), and its forward runs a twin of the same family at the
    # padded counts (outside the module tree: it owns no state).  Each forward hands the twin its parameters as
    # differentiable zero-padded functions of the real ones (so autograd returns the real parameters' gradients) and
    # its running statistics; padded channels have zero weights, bias and BatchNorm affine, so their activations are 0
    # and they add exact zeros to every real channel.  Running statistics are copied back after a training forward.
    def _twin_forward(self, x_t1, x_t2):
        tw, (maps, bufs) = self._twin_ready(x_t1.device)
        tw.train(self.training)
        for k, p in self.named_parameters():
            shape, m = maps[k]
            mod_name, _, attr = k.rpartition('.')
            object.__setattr__(tw.get_submodule(mod_name), attr, _scatter(p, shape, m))
        with torch.no_grad():
            for k, b in self.named_buffers():
                tb, m = bufs[k]
                if m and m[0] is not None:
                    tb.index_copy_(0, m[0], b)
                else:
                    tb.copy_(b)
        out = tw._forward(x_t1, x_t2)
        if self.training:
            with torch.no_grad():
                for k, b in self.named_buffers():
                    tb, m = bufs[k]
                    b.copy_(_gather(tb, m) if m else tb)
        return out

    def _twin_ready(self, dev):
        """(twin on `dev`, (parameter maps {name: (twin shape, per-dim positions)}, buffer maps {name: (twin buffer,
        positions)})), built on first use."""
        tw = self._twin
        if tw is None:
            import copy
            cfg = copy.deepcopy(self.cfg)
            if hasattr(cfg, 'defrost'):
                cfg.defrost()
            cfg.MODEL.TOPOLOGY = list(self._twin_topo)
            tw = type(self)(cfg)
            tw.conv_math = self.conv_math
            object.__setattr__(self, '_twin', tw)
            object.__setattr__(self, '_twin_maps', None)
        if next(tw.buffers()).device != torch.device(dev):
            tw.to(dev)  # buffers only: the twin's parameters are plain attributes, set per forward
            object.__setattr__(self, '_twin_maps', None)
        if self._twin_maps is None:
            tw_params = getattr(self, '_twin_shapes', None)
            if tw_params is None:  # first build: record the twin's parameter shapes (device-independent)
                tw_params = {k: tuple(v.shape) for k, v in tw.named_parameters()}
                object.__setattr__(self, '_twin_shapes', tw_params)
            for mod in tw.modules():  # from now on the twin's parameters are plain tensor attributes set per forward
                for k in list(mod._parameters):
                    v = mod._parameters.pop(k)
                    object.__setattr__(mod, k, v.detach())
            maps = {}
            mtype = str(self.cfg.MODEL.TYPE)
            for k, p in self.named_parameters():
                maps[k] = (tw_params[k], [_dim_map(r, q, dev, d == 1 and _concat_input(mtype, k))
                                          for d, (r, q) in enumerate(zip(p.shape, tw_params[k]))])
            bufs = {}
            tb = dict(tw.named_buffers())
            for k, b in self.named_buffers():
                if b.dim() == 1:
                    bufs[k] = (tb[k], [_dim_map(b.shape[0], tb[k].shape[0], dev)])
                else:
                    bufs[k] = (tb[k], [])
            object.__setattr__(self, '_twin_maps', (maps, bufs))
        return tw, self._twin_maps


def _ups_buffers(bufs, decoder, n_levels):
    """Per Up of `decoder` (up_seq order), the concat buffer the encoder wrote its skip into (or None)."""
    return [bufs[n_levels - 2 - k] for k in range(len(decoder.up_seq))]


def _stream(inc, encoder, decoder, x, nseg, training, siamese, head=None):
    """inc + encoder (+ Siamese diff) + decoder of one stream; returns (decoder output, features).  With `head` (the
    OutConv that is the decoder output's only reader) the first item is the head's logits (engine.run_decoder); with
    head='raw' it is the decoder's unmaterialised output for engine.run_heads."""
    n_levels = len(encoder.down_seq) + 1
    if siamese and engine.option('fuse_siamese_encoder'):  # networks.py:141-150, fused (engine.SiameseLevelFn)
        diffs, bufs = engine.run_siamese_encoder(inc, encoder, x, training,
                                                 engine.decoder_cat_channels(decoder, n_levels))
        feats = diffs[::-1]  # Encoder.forward returns the reversed list (networks.py:342)
        return engine.run_decoder(decoder, feats, training, _ups_buffers(bufs, decoder, n_levels), head=head), feats
    if not siamese and engine.option('fuse_plain_encoder'):  # each level's skip written into its concat buffer
        feats, bufs = engine.run_encoder(inc, encoder, x, nseg, training,
                                         engine.decoder_cat_channels(decoder, n_levels), with_buffers=True)
        feats = feats[::-1]
        return engine.run_decoder(decoder, feats, training, _ups_buffers(bufs, decoder, n_levels), head=head), feats
    feats = engine.run_encoder(inc, encoder, x, nseg, training)
    if siamese:
        feats = [engine.siamese_diff(f) for f in feats]
    feats = feats[::-1]
    return engine.run_decoder(decoder, feats, training, head=head), feats


def _fused_heads(cfg, heads) -> bool:
    """Whether a two-decoder model runs its heads as one engine.run_heads launch (engine option fuse_heads; at most 4
    output channels over all its heads, e.g. OUT_CHANNELS 1 for WhateverNet's three heads)."""
    return (engine.option('fuse_heads') and sum(o.conv.out_channels for o in heads) <= 4
            and all(o.conv.bias is not None for o in heads))


class UNet(_HipNet):
    def __init__(self, cfg):
        super().__init__(cfg)
        topology = cfg.MODEL.TOPOLOGY
        self.inc = InConv(cfg.MODEL.IN_CHANNELS * 2, topology[0], DoubleConv)
        self.encoder = Encoder(cfg)
        self.decoder = Decoder(cfg)
        self.outc = OutConv(topology[0], cfg.MODEL.OUT_CHANNELS)

    def _forward(self, x_t1, x_t2):
        x = engine.pack_stream(x_t1, x_t2)  # torch.cat((x_t1, x_t2), dim=1) (networks.py:74)
        out, _ = _stream(self.inc, self.encoder, self.decoder, x, 1, self.training, siamese=False, head=self.outc)
        return out  # self.outc(decoder output) (networks.py:77-78), fused into the decoder stage


class DualStreamUNet(_HipNet):
    def __init__(self, cfg):
        super().__init__(cfg)
        topology = cfg.MODEL.TOPOLOGY
        n1, n2 = _band_counts(cfg)
        self.inc_stream1 = InConv(2 * n1, topology[0], DoubleConv)
        self.encoder_stream1 = Encoder(cfg)
        self.decoder_stream1 = Decoder(cfg)
        self.inc_stream2 = InConv(2 * n2, topology[0], DoubleConv)
        self.encoder_stream2 = Encoder(cfg)
        self.decoder_stream2 = Decoder(cfg)
        self.outc = OutConv(2 * topology[0], cfg.MODEL.OUT_CHANNELS)

    def _forward(self, x_t1, x_t2):
        n1, _ = _band_counts(self.cfg)
        c = x_t1.shape[1]
        fused = _fused_heads(self.cfg, [self.outc])
        head = 'raw' if fused else None
        x1 = engine.pack_stream(x_t1, x_t2, 0, n1)
        d1, _ = _stream(self.inc_stream1, self.encoder_stream1, self.decoder_stream1, x1, 1, self.training, False, head)
        x2 = engine.pack_stream(x_t1, x_t2, n1, c - n1)
        d2, _ = _stream(self.inc_stream2, self.encoder_stream2, self.decoder_stream2, x2, 1, self.training, False, head)
        if fused:
            # self.outc(cat(x_stream1, x_stream2)) (networks.py:117-120): one launch over both decoders' last BatchNorm
            # + ReLU, no cat and no materialised decoder outputs
            return engine.run_heads([d1, d2], [(self.outc, (0, 1))])[0]
        return engine.run_head(self.outc, engine.cat_channels(d1, d2))


class SiameseUNet(_HipNet):
    def __init__(self, cfg):
        super().__init__(cfg)
        topology = cfg.MODEL.TOPOLOGY
        self.inc = InConv(cfg.MODEL.IN_CHANNELS, topology[0], DoubleConv)
        self.encoder = Encoder(cfg)
        self.decoder = Decoder(cfg)
        self.outc = OutConv(topology[0], cfg.MODEL.OUT_CHANNELS)

    def _forward(self, x_t1, x_t2):
        x = engine.pack_pair(x_t1, x_t2)
        out, _ = _stream(self.inc, self.encoder, self.decoder, x, 2, self.training, siamese=True, head=self.outc)
        return out  # self.outc(decoder output) (networks.py:152-153), fused into the decoder stage


class DualTaskSiameseUNet(_HipNet):
    # outc_sem_change is built (state_dict keys) but never called by forward (reference networks.py:174, 176-197;
    # assessment_semantics.py:34,117 calls it directly); parallel.wrap_ddp turns DDP's unused-parameter search on
    PARAMS_OUTSIDE_FORWARD = ('outc_sem_change',)

    def __init__(self, cfg):
        super().__init__(cfg)
        topology = cfg.MODEL.TOPOLOGY
        n_classes = cfg.MODEL.OUT_CHANNELS
        self.inc = InConv(cfg.MODEL.IN_CHANNELS, topology[0], DoubleConv)
        self.encoder = Encoder(cfg)
        self.decoder_change = Decoder(cfg)
        self.decoder_sem = Decoder(cfg)
        self.outc_change = OutConv(topology[0], n_classes)
        self.outc_sem = OutConv(topology[0], n_classes)
        self.outc_sem_change = OutConv(2, 1)  # present in the reference, unused by forward (networks.py:174)

    def _forward(self, x_t1, x_t2):
        b = x_t1.shape[0]
        x = engine.pack_pair(x_t1, x_t2)
        if engine.option('fuse_dualtask') and engine.option('pooled_bn_bwd'):
            return self._forward_fused(x, b)
        feats = engine.run_encoder(self.inc, self.encoder, x, 2, self.training)
        diffs = [engine.siamese_diff(f) for f in feats][::-1]
        # each decoder output feeds one head (networks.py:187-195): the heads run fused into the decoder stages
        out_change = engine.run_decoder(self.decoder_change, diffs, self.training, head=self.outc_change)
        f_t2 = [f[b:] for f in feats][::-1]
        out_sem_t2 = engine.run_decoder(self.decoder_sem, f_t2, self.training, head=self.outc_sem)
        f_t1 = [f[:b] for f in feats][::-1]
        out_sem_t1 = engine.run_decoder(self.decoder_sem, f_t1, self.training, head=self.outc_sem)
        return out_change, out_sem_t1, out_sem_t2

    def _forward_fused(self, x, b):
        """One pass per encoder level writes the difference into decoder_change's concat buffers and [f_t2; f_t1] into
        decoder_sem's (engine.DualTaskLevelFn); decoder_sem then runs both dates as one 2B batch whose BatchNorm
        segments are the two reference calls, t2 first (networks.py:190-195), or (engine option dt_sem_batched off) as
        two calls on the halves of the same buffers."""
        n_levels = len(self.encoder.down_seq) + 1
        diffs, sems, bufc, bufs = engine.run_dualtask_encoder(
            self.inc, self.encoder, x, self.training, engine.decoder_cat_channels(self.decoder_change, n_levels),
            engine.decoder_cat_channels(self.decoder_sem, n_levels))
        out_change = engine.run_decoder(self.decoder_change, diffs[::-1], self.training,
                                        _ups_buffers(bufc, self.decoder_change, n_levels), head=self.outc_change)
        sem_bufs = _ups_buffers(bufs, self.decoder_sem, n_levels)
        if engine.option('dt_sem_batched'):
            sem = engine.run_decoder(self.decoder_sem, sems[::-1], self.training, sem_bufs, head=self.outc_sem, nseg=2)
            return out_change, sem[b:], sem[:b]
        outs = []
        for lo in (0, b):  # t2 (images [0, b) of the semantic batch) first, then t1
            outs.append(engine.run_decoder(self.decoder_sem, [f[lo:lo + b] for f in sems[::-1]], self.training,
                                           [None if t is None else t[lo:lo + b] for t in sem_bufs],
                                           head=self.outc_sem))
        return out_change, outs[1], outs[0]


def _two_stream_heads(net, x1, x2, nseg: int, siamese: bool):
    """WhateverNet / WhateverNet2 (networks.py:226-263, 282-310): both streams, then outc_stream1(x_stream1),
    outc_stream2(x_stream2) and outc_fusion(cat(x_stream1, x_stream2)).  Fused (engine option fuse_heads): the three
    heads are one launch over both decoders' last BatchNorm + ReLU (engine.run_heads); else materialised outputs, a cat
    and three head launches."""
    heads = [(net.outc_fusion, (0, 1)), (net.outc_stream1, (0,)), (net.outc_stream2, (1,))]
    fused = _fused_heads(net.cfg, [h for h, _ in heads])
    head = 'raw' if fused else None
    d1, _ = _stream(net.inc_stream1, net.encoder_stream1, net.decoder_stream1, x1, nseg, net.training, siamese, head)
    d2, _ = _stream(net.inc_stream2, net.encoder_stream2, net.decoder_stream2, x2, nseg, net.training, siamese, head)
    if fused:
        out_fusion, out_stream1, out_stream2 = engine.run_heads([d1, d2], heads)
    else:
        out_stream1 = engine.run_head(net.outc_stream1, d1)
        out_stream2 = engine.run_head(net.outc_stream2, d2)
        out_fusion = engine.run_head(net.outc_fusion, engine.cat_channels(d1, d2))
    if net.training:
        return out_fusion, out_stream1, out_stream2
    return out_fusion


class WhateverNet(_HipNet):
    def __init__(self, cfg):
        super().__init__(cfg)
        topology = cfg.MODEL.TOPOLOGY
        n_classes = cfg.MODEL.OUT_CHANNELS
        n1, n2 = _band_counts(cfg)
        self.inc_stream1 = InConv(n1, topology[0], DoubleConv)
        self.encoder_stream1 = Encoder(cfg)
        self.decoder_stream1 = Decoder(cfg)
        self.outc_stream1 = OutConv(topology[0], n_classes)
        self.inc_stream2 = InConv(n2, topology[0], DoubleConv)
        self.encoder_stream2 = Encoder(cfg)
        self.decoder_stream2 = Decoder(cfg)
        self.outc_stream2 = OutConv(topology[0], n_classes)
        self.outc_fusion = OutConv(2 * topology[0], n_classes)

    def _forward(self, x_t1, x_t2):
        n1, _ = _band_counts(self.cfg)
        c = x_t1.shape[1]
        x1 = engine.pack_pair(x_t1, x_t2, 0, n1)
        x2 = engine.pack_pair(x_t1, x_t2, n1, c - n1)
        return _two_stream_heads(self, x1, x2, 2, True)


class WhateverNet2(_HipNet):
    def __init__(self, cfg):
        super().__init__(cfg)
        topology = cfg.MODEL.TOPOLOGY
        n_classes = cfg.MODEL.OUT_CHANNELS
        n1, n2 = _band_counts(cfg)
        self.inc_stream1 = InConv(2 * n1, topology[0], DoubleConv)
        self.encoder_stream1 = Encoder(cfg)
        self.decoder_stream1 = Decoder(cfg)
        self.outc_stream1 = OutConv(topology[0], n_classes)
        self.inc_stream2 = InConv(2 * n2, topology[0], DoubleConv)
        self.encoder_stream2 = Encoder(cfg)
        self.decoder_stream2 = Decoder(cfg)
        self.outc_stream2 = OutConv(topology[0], n_classes)
        self.outc_fusion = OutConv(2 * topology[0], n_classes)

    def _forward(self, x_t1, x_t2):
        n1, _ = _band_counts(self.cfg)
        c = x_t1.shape[1]
        x1 = engine.pack_stream(x_t1, x_t2, 0, n1)
        x2 = engine.pack_stream(x_t1, x_t2, n1, c - n1)
        return _two_stream_heads(self, x1, x2, 1, False)


# ------------------------------------------------------------------------------------------------
# Building blocks: the reference's attribute paths and parameters; forwards on the HIP kernels (NCHW in and out).
# ------------------------------------------------------------------------------------------------
class Encoder(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.cfg = cfg
        down_topo = cfg.MODEL.TOPOLOGY
        n_layers = len(down_topo)
        down_dict = OrderedDict()
        for idx in range(n_layers):
            in_dim = down_topo[idx]
            out_dim = down_topo[idx + 1] if idx != n_layers - 1 else down_topo[idx]
            down_dict[f'down{idx + 1}'] = Down(in_dim, out_dim, DoubleConv)
        self.down_seq = nn.ModuleDict(down_dict)

    def forward(self, x1):
        """[x1, down1(x1), down2(...), ...] reversed (networks.py:334-343)."""
        feats = [x1]
        for layer in self.down_seq.values():
            feats.append(layer(feats[-1]))
        feats.reverse()
        return feats


class Decoder(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.cfg = cfg
        topology = cfg.MODEL.TOPOLOGY
        n_layers = len(topology)
        up_topo = [topology[0]]
        for idx in range(n_layers):
            up_topo.append(topology[idx + 1] if idx != n_layers - 1 else topology[idx])
        up_dict = OrderedDict()
        for idx in reversed(range(n_layers)):
            x2_idx = idx - 1 if idx != 0 else idx
            up_dict[f'up{idx + 1}'] = Up(up_topo[idx] * 2, up_topo[x2_idx], DoubleConv)
        self.up_seq = nn.ModuleDict(up_dict)

    def forward(self, features):
        """Pops the deepest map off `features` (the caller's list, as the reference does) and runs the Up blocks
        against the rest (networks.py:375-382)."""
        x1 = features.pop(0)
        for idx, layer in enumerate(self.up_seq.values()):
            x1 = layer(x1, features[idx])
        return x1


class DoubleConv(nn.Module):
    '''(conv => BN => ReLU) * 2'''

    def __init__(self, in_ch, out_ch):
        super().__init__()
        self.conv = nn.Sequential(
            nn.Conv2d(in_ch, out_ch, 3, padding=1),
            nn.BatchNorm2d(out_ch),
            nn.ReLU(inplace=True),
            nn.Conv2d(out_ch, out_ch, 3, padding=1),
            nn.BatchNorm2d(out_ch),
            nn.ReLU(inplace=True),
        )

    def forward(self, x):
        return _block(self, x, maxpool=False)


def _block(dc: DoubleConv, x, maxpool: bool):
    """DoubleConv (networks.py:386-402), behind MaxPool2d(2) for Down (415-426), on the engine's block Function.  A
    source whose channels are not a multiple of 8 is zero-padded (its input gradient is then not available)."""
    cin = x.shape[1]
    cp = engine.pad_in(cin) if cin % 8 else cin
    y = engine.run_block(dc, engine.to_nhwc(x, cp), dc.training, maxpool=maxpool)
    return engine.to_nchw(y)


class InConv(nn.Module):
    def __init__(self, in_ch, out_ch, conv_block):
        super().__init__()
        self.conv = conv_block(in_ch, out_ch)

    def forward(self, x):
        return self.conv(x)


class Down(nn.Module):
    def __init__(self, in_ch, out_ch, conv_block):
        super().__init__()
        self.mpconv = nn.Sequential(nn.MaxPool2d(2), conv_block(in_ch, out_ch))

    def forward(self, x):
        return _block(self.mpconv[1], x, maxpool=True)


class Up(nn.Module):
    def __init__(self, in_ch, out_ch, conv_block):
        super().__init__()
        self.up = nn.ConvTranspose2d(in_ch // 2, in_ch // 2, 2, stride=2)
        self.conv = conv_block(in_ch, out_ch)

    def forward(self, x1, x2):
        """ConvT(x1), F.pad to x2's size, cat([x2, up], 1), DoubleConv (networks.py:436-451)."""
        y = engine.run_ups([self], [engine.to_nhwc(x1), engine.to_nhwc(x2)], self.training)
        return engine.to_nchw(y)


class OutConv(nn.Module):
    def __init__(self, in_ch, out_ch):
        super().__init__()
        self.conv = nn.Conv2d(in_ch, out_ch, 1)

    def forward(self, x):
        return engine.run_head(self, engine.to_nhwc(x))
