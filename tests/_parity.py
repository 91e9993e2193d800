"""Shared parity machinery of the -m gpu model tests (test infrastructure, imports the oracle).

Gradients: branch matching.  A training step's gradient is a piecewise-linear function's: every ReLU decision
(BatchNorm output > 0) and every MaxPool2d argmax picks a branch, and a pre-activation within rounding of the kink
(or a near-tie in a pooling window) is decided by the last bits of the forward -- any two fp32-class implementations
(the reference on CPU, the oracle, x3, h2) may take different branches there, and one such pixel moves upstream
weight gradients by up to a few percent.  BranchMatch reads the decisions the GPU forward actually took
(engine.trace_bn: every BatchNorm's conv output and coefficients) and the oracle follows them (siamese_oracle.BRANCH),
so branch_matched_reference() returns the fp64 gradient of the SAME branch: the difference to the GPU's gradient is
pure arithmetic error and every tensor is held to the strict bar, with no exemptions.

The reference's own fp32 gradients (the fixtures) took their own branches; they pin the oracle in
tests/test_oracle_golden.py, and the GPU tests check them loosely (norm-wise) beside the strict branch-matched bar.
"""
from __future__ import annotations

import contextlib
from collections import namedtuple

import numpy as np
import torch
import torch.nn.functional as F

KINK_REL = 1e-5
KINK_MAX_ERR = 3e-2
# Largest distance (max-relative) a GPU pre-activation may have from the branch-matched oracle's and still be adopted.
# h2 / x3 forwards sit at 1e-6-class distances (fp32 arithmetic); the guard leaves one decade of margin over the
# kink band, and every adopted decision is bounded by the band itself (BranchMatch.__call__).
MATCH_MAX_REL = 1e-4
_CONV2D = F.conv2d

Kink = namedtuple('Kink', 'key rel occ mask')


def rel(a, b) -> float:
    a = torch.as_tensor(a).detach().double().cpu()
    b = torch.as_tensor(b).detach().double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


def record_kinks(model, P, B, batch, ocfg, dtype=torch.float64, kink_rel=KINK_REL):
    """[Kink(BatchNorm key, min|z| / max|z|, occurrence, element mask)] of the oracle forward's kink-ambiguous
    pre-activations."""
    from oracle import siamese_oracle as O
    Pd = {k: v.detach().to(dtype) for k, v in P.items()}
    Bd = {k: (v.to(dtype) if v.is_floating_point() else v.clone()) for k, v in B.items()}
    O.RECORD = []
    try:
        with torch.no_grad():
            O.forward(model, Pd, Bd, batch['x_t1'].to(dtype), batch['x_t2'].to(dtype), ocfg, True)
        rec = O.RECORD
    finally:
        O.RECORD = None
    out, occ = [], {}
    for k, z in rec:
        o = occ[k] = occ.get(k, -1) + 1
        thr = kink_rel * float(z.abs().max())
        if float(z.abs().min()) < thr:
            out.append(Kink(k, float(z.abs().min() / z.abs().max()), o, z.abs() < thr))
    return out


def _is_pre_bn_bias(k: str) -> bool:
    return k.endswith('conv.0.bias') or k.endswith('conv.3.bias')


def check_gradients(got: dict, ref: dict, order: list, bars: dict, kinks: list) -> list:
    """got / ref: name -> tensor; order: parameter names in forward (named_parameters) order; bars: name -> the
    relative max-norm bar.  Without branch matching (the multi-rank test): a tensor over its bar is accepted only
    upstream of the latest kink-ambiguous BatchNorm output (`kinks`, record_kinks) and within KINK_MAX_ERR.
    Returns the list of failures (empty = pass)."""
    pos = {k: i for i, k in enumerate(order)}
    last_kink = max((pos.get(kk[0] + '.weight', -1) for kk in kinks), default=-1)
    bad = []
    for k in order:
        if k not in ref or _is_pre_bn_bias(k):
            continue
        g, r = got[k].detach().double().cpu(), ref[k].detach().double().cpu()
        err = ((g - r).abs().max() / r.abs().max().clamp_min(1e-30)).item()
        if err <= bars[k]:
            continue
        ok = bool(kinks) and pos[k] <= last_kink and err < KINK_MAX_ERR
        why = 'upstream of the latest kink' if pos[k] <= last_kink else 'DOWNSTREAM of every kink'
        print(f'{k:60s} err {err:.2e} > bar {bars[k]:.2e}; {why}; {"accepted" if ok else "FAIL"}')
        if not ok:
            bad.append((k, err))
    if kinks:
        print('kink-ambiguous pre-activations:', [(kk[0], kk[1]) for kk in kinks])
    return bad


class BranchMatch:
    """siamese_oracle.BRANCH from a GPU forward's engine.trace_bn() record.

    Per BatchNorm module and segment the GPU's pre-activation z = fma(y, scale, shift) is formed in fp64 (the product
    of two fp32 values is exact there, so z > 0 is exactly the GPU's fmaf(...) > 0 decision); an oracle call is
    matched to the batch chunk of that module's records closest to its own pre-activation (model-agnostic: the GPU
    batches the Siamese branches and the decoder_sem runs of the dual-task model, the oracle calls them one by one).
    The activation returned for the pooling argmax is relu(z) rounded to fp32, the values the GPU pooled."""

    def __init__(self, trace, module, max_rel: float = MATCH_MAX_REL, kink_rel: float = KINK_REL):
        """module: the model (its named_modules name the traced BatchNorms), or a dict {id(bn): name}.

        Every adopted decision is bounded: a ReLU decision of the GPU that differs from the sign of the oracle's own
        pre-activation must lie in the kink band |z_oracle| <= kink_rel * max|z_oracle|, and a 2x2 window whose GPU
        argmax differs from the argmax of the oracle's own activation must be a near-tie (the two candidates' oracle
        activations within kink_rel * max|z_oracle|).  Anything else is a wrong branch, not a rounding choice, and
        raises.  The counts are kept (flips, pool_flips) and printed."""
        if isinstance(module, dict):
            names = module
        else:  # a model off the granule of 8 runs a padded twin (utils/networks.py): its BatchNorms, same names
            names = {id(m): n for n, m in module.named_modules()}
            twin = getattr(module, '_twin', None)
            if twin is not None:
                names.update({id(m): n for n, m in twin.named_modules()})
        self.segs: dict = {}  # key -> [(y fp32 NHWC of one segment, scale, shift)], z formed per call (memory)
        for bn, y, scale, shift, nseg in trace:
            n, c = y.shape[0], y.shape[3]
            per = n // nseg
            y32 = y.detach().cpu()
            sc = scale.detach().double().cpu().view(nseg, c)
            sh = shift.detach().double().cpu().view(nseg, c)
            for s in range(nseg):
                self.segs.setdefault(names[id(bn)], []).append((y32[s * per:(s + 1) * per], sc[s], sh[s]))
        self.max_rel = max_rel
        self.kink_rel = kink_rel
        self.worst = 0.0
        self.calls = 0
        self.flips = 0  # ReLU decisions adopted from the GPU against the oracle's own sign (all inside the kink band)
        self.pool_flips = 0  # 2x2 windows whose adopted argmax differs from the oracle's own (all near-ties)
        self.elements = 0
        self.windows = 0

    def __call__(self, key, y):
        nb = y.shape[0]
        yd = y.detach().double()
        den = yd.abs().max().clamp_min(1e-30)
        best, best_d = None, float('inf')
        c = y.shape[1]
        for y32, sc, sh in self.segs[key]:  # a padded twin's channels: the real ones are the prefix
            if tuple(y32.shape[1:3]) != (y.shape[2], y.shape[3]) or y32.shape[3] < c or y32.shape[0] % nb:
                continue
            for i in range(0, y32.shape[0], nb):
                z = (y32[i:i + nb, :, :, :c].double() * sc[:c] + sh[:c]).permute(0, 3, 1, 2)
                d = ((z - yd).abs().max() / den).item()
                if d < best_d:
                    best, best_d = z.contiguous(), d
        if best is None or best_d > self.max_rel:
            raise AssertionError(f'{key}: no GPU pre-activation within {self.max_rel} of the oracle\'s ({best_d:.2e})')
        self.worst = max(self.worst, best_d)
        self.calls += 1
        band = self.kink_rel * float(den)
        mask = best > 0
        flip = mask != (yd > 0)
        nflip = int(flip.sum())
        if nflip:
            far = flip & (yd.abs() > band)
            if bool(far.any()):
                raise AssertionError(
                    f'{key}: {int(far.sum())} GPU ReLU decisions differ from the oracle\'s outside the kink band '
                    f'(|z| up to {float(yd.abs()[far].max() / den):.2e} of max, band {self.kink_rel:.0e})')
        self.flips += nflip
        self.elements += flip.numel()
        a = torch.relu(best.float())
        if y.shape[2] >= 2 and y.shape[3] >= 2:  # a MaxPool2d(2) may follow: its window argmaxes are adopted too
            from oracle.siamese_oracle import _windows
            wg = _windows(a.double())
            wo = _windows(torch.relu(yd))
            ig, io = wg.argmax(-1, keepdim=True), wo.argmax(-1, keepdim=True)
            diff = (ig != io).squeeze(-1)
            npf = int(diff.sum())
            if npf:
                gap = (wo.gather(-1, io) - wo.gather(-1, ig)).squeeze(-1)[diff]
                if float(gap.max()) > band:
                    raise AssertionError(
                        f'{key}: {int((gap > band).sum())} pooling windows whose GPU argmax is not a near-tie of the '
                        f'oracle\'s (gap up to {float(gap.max() / den):.2e} of max, band {self.kink_rel:.0e})')
            self.pool_flips += npf
            self.windows += diff.numel()
        return mask, a.to(y.dtype)

    def summary(self) -> str:
        return (f'{self.calls} BatchNorm outputs matched, worst pre-activation distance {self.worst:.2e} '
                f'(guard {self.max_rel:.0e}); ReLU decisions adopted against the oracle\'s sign: {self.flips} of '
                f'{self.elements} (all within {self.kink_rel:.0e} of max); pooling argmaxes adopted: {self.pool_flips} '
                f'of {self.windows} windows (all near-ties)')


def branch_matched_reference(model_type, P, batch, ocfg, trace, module, loss_fn, training=True, buffers=None):
    """(outputs, loss, {name: grad}) of the fp64 oracle following the branches of the GPU forward recorded in
    `trace` (engine.trace_bn()).  loss_fn(outputs, batch) -> scalar (e.g. siamese_oracle.step_loss).  `buffers`
    (fresh ones by default) are converted to fp64, updated by the forward, and copied back."""
    from oracle import siamese_oracle as O
    Pd = {k: v.detach().double().clone().requires_grad_(True) for k, v in P.items()}
    if buffers is None:
        buffers = O.fresh_buffers(O.param_shapes(model_type, ocfg))
    Bd = {k: (v.double() if v.is_floating_point() else v.clone()) for k, v in buffers.items()}
    bt = {k: (v.detach().cpu().double() if v.is_floating_point() else v.detach().cpu()) for k, v in batch.items()}
    bm = BranchMatch(trace, module)
    O.BRANCH = bm
    try:
        out = O.forward(model_type, Pd, Bd, bt['x_t1'], bt['x_t2'], ocfg, training)
    finally:
        O.BRANCH = None
    with torch.no_grad():
        for k, v in Bd.items():
            buffers[k].copy_(v)
    loss = loss_fn(out, bt)
    loss.backward()
    print(f'branch matching: {bm.summary()}')
    return out, loss, {k: v.grad for k, v in Pd.items() if v.grad is not None}


def check_branch_matched(got: dict, ref: dict, order: list, bar: float) -> list:
    """Every tensor (pre-BatchNorm conv biases aside: true gradient 0) within `bar` max-relative of the
    branch-matched fp64 gradient.  Returns the failures; prints the worst tensor."""
    bad, worst = [], (None, 0.0)
    for k in order:
        if k not in ref or _is_pre_bn_bias(k):
            continue
        e = rel(got[k], ref[k])
        worst = max(worst, (k, e), key=lambda t: t[1])
        if not e <= bar:
            bad.append((k, e))
    print(f'gradients vs the branch-matched fp64 oracle: worst {worst[1]:.2e} ({worst[0]}), bar {bar:.0e}')
    return bad


def rel_l2(a, b) -> float:
    a = torch.as_tensor(a).detach().double().cpu()
    b = torch.as_tensor(b).detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def mask_mismatch(out, ref, tol=1e-4) -> int:
    """Change-mask (logit > 0, utils/metrics.py:26) pixels that differ outside the |ref| < tol * max band."""
    out = np.asarray(out, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    band = np.abs(ref) < tol * np.abs(ref).max()
    return int((((out > 0) != (ref > 0)) & ~band).sum())


def r16(t):
    return t.to(torch.bfloat16).float()


# Accumulation type of the bf16-emulating convs: double by default; bf16_conv_oracle(torch.float32) at the shipped
# batches (a bf16 x bf16 product is exact in fp32 as in double, so only the summation rounding differs -- the GPU's
# own accumulation is fp32 -- at half the CPU time of double).
_ACC16 = [torch.float64]


class _Conv16(torch.autograd.Function):
    """A 3x3 conv with the bf16 kernels' arithmetic: bf16-rounded operands in forward, data-grad and weight-grad,
    exact products, fp32 (here double, or _ACC16) accumulation; the output and the data grad rounded to bf16 as bf16
    storage (engine.act_storage_for) keeps them in HBM."""

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        acc = _ACC16[0]
        return r16(_CONV2D(r16(x).to(acc), r16(w).to(acc), None, padding=1).float() + b[None, :, None, None])

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        acc = _ACC16[0]
        g16 = r16(gy).to(acc)
        gx = r16(torch.nn.grad.conv2d_input(x.shape, r16(w).to(acc), g16, padding=1).float())
        gw = torch.nn.grad.conv2d_weight(r16(x).to(acc), w.shape, g16, padding=1).float()
        return gx, gw, gy.sum((0, 2, 3))


_CONVT2D = F.conv_transpose2d


class _ConvT16(torch.autograd.Function):
    """A ConvTranspose2d(k=2, s=2) with the bf16 configs' arithmetic (libscd: the gather kernel's and the generic
    weight grad's bf16 instances): the forward (fwd16) and the data grad (bwd16, where the gather kernel takes them)
    and the weight grad (always) on bf16-rounded operands, exact products, fp32 (here double) accumulation."""

    @staticmethod
    def forward(ctx, x, w, b, fwd16, bwd16):
        ctx.save_for_backward(x, w)
        ctx.bwd16 = bwd16
        xx, ww = (r16(x), r16(w)) if fwd16 else (x, w)
        acc = _ACC16[0]
        return _CONVT2D(xx.to(acc), ww.to(acc), None, stride=2).float() + b[None, :, None, None]

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        gg, ww = (r16(gy), r16(w)) if ctx.bwd16 else (gy, w)
        acc = _ACC16[0]
        gx = _CONV2D(gg.to(acc), ww.to(acc), None, stride=2).float()  # the transpose of the ConvT
        with torch.enable_grad():
            wr = w.detach().to(acc).requires_grad_(True)
            gw, = torch.autograd.grad(_CONVT2D(r16(x.detach()).to(acc), wr, None, stride=2), wr, r16(gy).to(acc))
        return gx, gw.float(), gy.sum((0, 2, 3)), None, None


def convT_bf16(x, w, b=None, stride=1, padding=0, *a, **k):
    """F.conv_transpose2d(k=2, s=2) with the bf16 configs' arithmetic: forward and data grad in bf16 where libscd's
    gather kernel takes the launch (forward: in-channels % 32, 4 x out-channels % 64; data grad: out-channels % 32,
    in-channels % 64), fp32 otherwise; the weight grad in bf16."""
    if tuple(w.shape[2:]) == (2, 2) and stride == 2 and padding == 0 and not a and not k:
        fwd16 = w.shape[0] % 32 == 0 and w.shape[1] % 16 == 0
        bwd16 = w.shape[1] % 32 == 0 and w.shape[0] % 64 == 0
        return _ConvT16.apply(x, w, b if b is not None else w.new_zeros(w.shape[1]), fwd16, bwd16)
    return _CONVT2D(x, w, b, stride, padding, *a, **k)


@contextlib.contextmanager
def bf16_conv_oracle(accumulate=torch.float64):
    """Inside: every 3x3 conv the bf16 kernels take (source channels a multiple of 32, or an input layer of at most
    16 bands, zero-padded to the 16-channel kernels) runs through _Conv16, every ConvTranspose through convT_bf16;
    the rest stays fp32.  `accumulate`: the emulated convs' summation type (see _ACC16)."""
    prev_acc, _ACC16[0] = _ACC16[0], accumulate
    def conv(x, w, b=None, stride=1, padding=0, *a, **k):
        if (w.shape[2:] == (3, 3) and (w.shape[1] % 32 == 0 or w.shape[1] <= 16) and stride == 1
                and padding == 1):
            return _Conv16.apply(x, w, b)
        return _CONV2D(x, w, b, stride, padding, *a, **k)

    F.conv2d = conv
    F.conv_transpose2d = convT_bf16
    try:
        yield
    finally:
        F.conv2d = _CONV2D
        F.conv_transpose2d = _CONVT2D
        _ACC16[0] = prev_acc


def record_arith(monkeypatch, dev):
    """Wrap hip.conv_igemm / hip.conv_wgrad to record, per launch, (kind, src.c, n_out/rows, ntaps, arithmetic, the
    arithmetic it would have with a bound on every operand)."""
    from multimodal_siamese_cd_amd import hip
    seen = []
    orig_igemm, orig_wgrad = hip.conv_igemm, hip.conv_wgrad
    one = torch.ones(1, device=dev)

    def igemm(src, out_h, out_w, stride, taps, wpk, n_out, bias, dst, store_mode=0, **kw):
        a = hip.igemm_arith(src, out_h, out_w, stride, taps, wpk, n_out, dst, store_mode, src_bound=kw.get('src_bound'))
        b = hip.igemm_arith(src, out_h, out_w, stride, taps, wpk, n_out, dst, store_mode, src_bound=one)
        seen.append(('igemm', src.c, n_out, len(taps[0]), a, b))
        return orig_igemm(src, out_h, out_w, stride, taps, wpk, n_out, bias, dst, store_mode, **kw)

    def wgrad(d, slabs):
        e = hip.WGRAD.from_buffer_copy(d)
        e.rows_bound = e.src_bound = one.data_ptr()
        seen.append(('wgrad', d.src.c, d.rows.c, d.ntaps, hip.wgrad_arith(d), hip.wgrad_arith(e)))
        return orig_wgrad(d, slabs)

    monkeypatch.setattr(hip, 'conv_igemm', igemm)
    monkeypatch.setattr(hip, 'conv_wgrad', wgrad)
    return seen
