"""Throughput benchmark of the Siamese U-Net training step on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config baseline_siamese] [--batch B]
                    [--math h2|x3|x5|bf16|f32]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

One step = zero_grad -> SiameseUNet forward (HIP) -> power_jaccard_loss -> backward (HIP) -> AdamW step,
on synthetic 256x256 SAR(2)+optical(3) pairs generated on the device (weak scaling: every rank draws its
own batch).  Rank 0 prints ONE JSON line; `value` is pairs/s of the whole job (all ranks' pairs / max rank time).

Conv arithmetic.  A model carries it per launch descriptor (no library mode, no environment switch): a config with
MODEL.PRECISION fp32 runs h2 (the default: each fp32 operand as a two-term fp16 split after power-of-two scaling,
three fp16 MFMA products, fp32 accumulation; fp32-class results), MODEL.PRECISION bf16 runs bf16; `--math` overrides
it (x3: exact three-term bf16 split, six products; x5: x3 less one product; f32: fp32 MFMA).  `dtype` names the
arithmetic: "f32 (h2 split-fp16)" for the default.

Measurement extras (rank 0, after the timed region):
  roofline      the MFMA conv kernels (every conv launch of one step) bracketed by HIP events on the launch
                stream: algorithmic conv FLOPs per step / summed kernel time.  The peak is each launch's own
                matrix-core ceiling (the library reports every launch's arithmetic: scd_igemm_arith /
                scd_wgrad_arith), combined flop-weighted harmonically:
                  - h2: fp16 dense 2516.8 / 3 products = 838.9 fp32-equivalent TFLOP/s;
                  - x3: bf16 dense 2516.8 / 6 products = 419.5; x5: / 5 = 503.4;
                  - bf16: bf16 dense 2516.8; fp32 MFMA: 157.3 (MI355X_MICROARCH.md).
                by_class / dominant_kernel split the same events per kernel family.
  step_roofline the survey's whole-step formula: 3x3-stack train FLOP/pair x pairs/s/GPU over the
                peak of the arithmetic the step runs (h2 838.9 for the default), with the nominal fp32-MFMA ratio
                beside it, labelled as such.
  cpu_baseline  the CPU oracle (oracle/siamese_oracle.py, torch fp32 on every host core this process may use)
                running the same training step on bounded samples at bs=2 and bs=8, 256x256.
  distributed   under torchrun: process-group backend, world size, per-rank ms per step (min / max) and the exposed
                gradient all-reduce on rank 0 (HIP events: from the last parameter gradient the backward produces to
                the end of backward, where DDP's reducer makes the compute stream wait for the last bucket).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from multimodal_siamese_cd_amd import engine, hip, parallel, trainers  # noqa: E402
from multimodal_siamese_cd_amd.utils import datasets, experiment_manager, networks  # noqa: E402

FP32_MFMA_PEAK_TFLOPS = 157.3
BF16_MFMA_PEAK_TFLOPS = 16 * FP32_MFMA_PEAK_TFLOPS  # dense, MI355X_MICROARCH.md (1/16 ratio)
X3_PEAK_TFLOPS = BF16_MFMA_PEAK_TFLOPS / 6           # six bf16 products per fp32 multiply-add
H2_PEAK_TFLOPS = BF16_MFMA_PEAK_TFLOPS / 3           # three fp16 products (fp16 dense = bf16 dense)
HBM_PEAK_TBS = 8.0  # HBM3E, MI355X_MICROARCH.md
PEAKS = {'f32': FP32_MFMA_PEAK_TFLOPS, 'x3': X3_PEAK_TFLOPS, 'x5': BF16_MFMA_PEAK_TFLOPS / 5,
         'bf16': BF16_MFMA_PEAK_TFLOPS, 'h2': H2_PEAK_TFLOPS}
METRIC = "image-pairs/sec training step, 256×256 SAR+optical Siamese U-Net, 1/2/4/8 MI355X"


def conv_flops(cfg, batch: int, size: int):
    """Algorithmic train FLOPs per step: 2*M*N*K per conv for fwd, data-grad (not for the input layer) and
    weight-grad; 3x3 stack and ConvTranspose counted separately."""
    topo = list(cfg.MODEL.TOPOLOGY)
    cin = cfg.MODEL.IN_CHANNELS
    L = len(topo)
    ch = [topo[0]] + [topo[i + 1] if i != L - 1 else topo[i] for i in range(L)]
    f3 = 0.0
    fT = 0.0
    n_enc = 2 * batch  # Siamese: both branches through the shared encoder
    for lvl in range(L + 1):
        hw = (size >> lvl) ** 2
        c_in = cin if lvl == 0 else ch[lvl - 1]
        for k, (a, b) in enumerate(((c_in, ch[lvl]), (ch[lvl], ch[lvl]))):
            fwd = 2.0 * n_enc * hw * b * 9 * a
            f3 += fwd * (2 if (lvl == 0 and k == 0) else 3)
    for idx in reversed(range(L)):  # decoder up{idx+1}
        hw = (size >> idx) ** 2
        c = ch[idx]
        out = ch[idx - 1] if idx != 0 else ch[0]
        fT += 3 * 2.0 * batch * (hw // 4) * (4 * c) * c
        f3 += 3 * 2.0 * batch * hw * out * 9 * (2 * c)
        f3 += 3 * 2.0 * batch * hw * out * 9 * out
    return f3, fT


def kernel_class(kind: str, ntaps: int, src_c: int) -> str:
    """The kernel family a conv launch runs on: 3x3 forward / data grad (igemm_halo16_x3), 3x3 weight grad
    (wgrad_halo16_x3), the 16-channel input layer (igemm / wgrad_halo16_c16), ConvTranspose (gather16 / generic)."""
    if ntaps == 9:
        return f"{kind}_3x3_input_layer" if src_c == 16 else f"{kind}_3x3"
    return f"{kind}_convT"


class KernelTimer:
    """HIP-event brackets around every MFMA conv launch (on torch's current stream, where libscd launches)."""

    def __init__(self):
        self.events = []
        self.active = False
        self._igemm = hip.conv_igemm
        self._wgrad = hip.conv_wgrad

    def install(self):
        timer = self

        def igemm(src, out_h, out_w, stride, taps, wpk, n_out, *a, **k):
            if not timer.active:
                return timer._igemm(src, out_h, out_w, stride, taps, wpk, n_out, *a, **k)
            arith = hip.igemm_arith(src, out_h, out_w, stride, taps, wpk, n_out, a[1] if len(a) > 1 else k['dst'],
                                    a[2] if len(a) > 2 else k.get('store_mode', 0), src_bound=k.get('src_bound'))
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            r = timer._igemm(src, out_h, out_w, stride, taps, wpk, n_out, *a, **k)
            e.record()
            flops = 2.0 * src.n * out_h * out_w * n_out * len(taps[0]) * src.c
            dst = a[1] if len(a) > 1 else k['dst']
            alg = hip.igemm_alg_bytes(src, out_h, out_w, taps, n_out, dst, arith,
                                      k['bn_bwd'][0] if k.get('bn_bwd') is not None else None)
            timer.events.append(('igemm', s, e, flops, arith, kernel_class('igemm', len(taps[0]), src.c), alg))
            return r

        def wgrad(d, slabs):
            if not timer.active:
                return timer._wgrad(d, slabs)
            arith = hip.wgrad_arith(d)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            r = timer._wgrad(d, slabs)
            e.record()
            flops = 2.0 * d.rows.n * d.rows.h * d.rows.w * d.rows.c * d.ntaps * d.src.c
            alg = hip.wgrad_alg_bytes(d, slabs.numel() * slabs.element_size())
            timer.events.append(('wgrad', s, e, flops, arith, kernel_class('wgrad', d.ntaps, d.src.c), alg))
            return r

        hip.conv_igemm = igemm
        hip.conv_wgrad = wgrad

    def summary(self):
        torch.cuda.synchronize()
        out = {}
        for name, s, e, *_ in self.events:
            n, t = out.get(name, (0, 0.0))
            out[name] = (n + 1, t + s.elapsed_time(e))
        return out

    def by_class(self, reps):
        """Per kernel class (kernel_class): launches, ms, FLOPs per step, TFLOP/s and the fraction of that class's
        flop-weighted arithmetic peak; the class with the most time is the step's dominant kernel."""
        out = {}
        for _, s, e, fl, arith, cls, _alg in self.events:
            c = out.setdefault(cls, {'n': 0, 'ms': 0.0, 'flop': 0.0, 'tpeak': 0.0})
            c['n'] += 1
            c['ms'] += s.elapsed_time(e)
            c['flop'] += fl
            c['tpeak'] += fl / (PEAKS[arith] * 1e12)
        res = {}
        for cls, c in out.items():
            ach = c['flop'] / (c['ms'] * 1e-3) / 1e12
            peak = c['flop'] / c['tpeak'] / 1e12
            res[cls] = {"launches_per_step": c['n'] // reps, "ms_per_step": round(c['ms'] / reps, 3),
                        "tflop_per_step": round(c['flop'] / reps / 1e12, 4), "achieved": round(ach, 2),
                        "peak": round(peak, 1), "frac": round(ach / peak, 4)}
        return res

    def peak(self):
        """Harmonic flop-weighted matrix-core peak of the timed launches (TFLOP/s) and each arithmetic's share."""
        f = sum(ev[3] for ev in self.events)
        t = sum(ev[3] / (PEAKS[ev[4]] * 1e12) for ev in self.events)
        share = {m: round(sum(ev[3] for ev in self.events if ev[4] == m) / f, 4) for m in PEAKS}
        return f / t / 1e12, {m: v for m, v in share.items() if v > 0}

    def launched_flops(self, reps):
        return sum(ev[3] for ev in self.events) / reps

    def alg_bytes(self, reps):
        """Algorithmic bytes of the conv launches per step: every operand read once, every output written once (src +
        dst + split weights for igemm, dY + X + slabs for wgrad, + the y a fused BatchNorm transform reads and the dy a
        weight grad forming a BatchNorm backward stores)."""
        return sum(ev[6] for ev in self.events) / reps


def host_cores() -> tuple:
    """(cores this process may run on: the CPU affinity set, capped by a cgroup CPU quota; os.cpu_count(); model)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, 'sched_getaffinity') else (os.cpu_count() or 1)
    try:
        with open('/sys/fs/cgroup/cpu.max') as f:
            quota, period = f.read().split()[:2]
        if quota != 'max':
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    model = 'unknown'
    try:
        with open('/proc/cpuinfo') as f:
            for line in f:
                if line.startswith('model name'):
                    model = line.split(':', 1)[1].strip()
                    break
    except OSError:
        pass
    return n, os.cpu_count(), model


def cpu_baseline(cfg, batches=(2, 8), min_seconds=(8.0, 6.0), size: int = 256):
    """The CPU oracle (torch fp32 on every host core this process may use) running the same training step on bounded
    samples, one per batch size (bs=2 and bs=8 at 256x256): whole steps after one warm-up until
    `min_seconds` of CPU work have been timed (at least 2 steps).  `value` is the larger batch's rate."""
    from oracle import siamese_oracle as O

    threads, ncpu, model = host_cores()
    torch.set_num_threads(threads)
    ocfg = dict(TOPOLOGY=list(cfg.MODEL.TOPOLOGY), IN_CHANNELS=cfg.MODEL.IN_CHANNELS, OUT_CHANNELS=1,
                S1_BANDS=list(cfg.DATALOADER.S1_BANDS), S2_BANDS=list(cfg.DATALOADER.S2_BANDS))
    mtype = cfg.MODEL.TYPE
    shapes = O.param_shapes(mtype, ocfg)
    by_batch, notes = {}, []
    for batch, tmin in zip(batches, min_seconds):
        P = {k: v.requires_grad_(True) for k, v in O.deterministic_params(shapes, 7).items()}
        B = O.fresh_buffers(shapes)
        b = O.synthetic_batch(ocfg, batch, size, 8)
        opt = torch.optim.AdamW(list(P.values()), lr=1e-4, weight_decay=0.01)

        def step():
            opt.zero_grad()
            out = O.forward(mtype, P, B, b['x_t1'], b['x_t2'], ocfg, True)
            loss = O.step_loss(mtype, out, b, 0.5)
            loss.backward()
            opt.step()

        step()  # warm-up
        t0 = time.perf_counter()
        steps = 0
        while steps < 2 or time.perf_counter() - t0 < tmin:
            step()
            steps += 1
        dt = time.perf_counter() - t0
        by_batch[str(batch)] = round(batch * steps / dt, 4)
        notes.append(f"bs={batch}: {steps} steps in {dt:.1f} s")
    return {"value": by_batch[str(batches[-1])], "unit": "image-pairs/s", "cores": threads, "kind": "port",
            "by_batch": by_batch, "cpu_model": model, "os_cpu_count": ncpu,
            "sample": f"timed training steps (after 1 warm-up each) of the CPU oracle ({mtype}), {size}x{size}, "
                      f"{cfg.MODEL.IN_CHANNELS}-ch, TOPOLOGY {list(cfg.MODEL.TOPOLOGY)}, fp32, torch "
                      f"{torch.__version__}, {threads} threads (the cores this process may use; os.cpu_count() "
                      f"{ncpu}); " + '; '.join(notes)}


def _conv_family(name: str):
    """igemm / wgrad (the conv kernels), other (libscd's non-conv kernels: BatchNorm, pool / difference, head, loss,
    packing, reductions) or torch (everything else in the step: the fused AdamW, torch's foreach adds)."""
    n = name.split('(')[0].replace('void ', '').replace('scd::', '').strip()
    if n.startswith('igemm'):
        return 'igemm'
    if n.startswith(('wgrad_halo', 'wgrad_x3', 'wgrad_f32')):
        return 'wgrad'
    return 'other' if 'scd::' in name else 'torch'



def live_traffic(args, batch: int, size: int, timeout_s: int = 180):
    """The conv kernels' HBM-side traffic per step, measured now: two child processes run 3 steps of this workload
    (1 warm-up + 2) under `rocprofv3 --pmc FETCH_SIZE` and `--pmc WRITE_SIZE` (separate passes, MI355X_MICROARCH.md
    HBM); FETCH_SIZE is doubled (the gfx950 correction for 16-byte-per-lane streaming reads), both are KiB.  Returns
    {bytes_per_step, by_family, source} or raises."""
    import csv
    import shutil
    import subprocess
    import tempfile
    prof = shutil.which('rocprofv3') or '/opt/rocm/bin/rocprofv3'
    if not os.path.exists(prof):
        raise RuntimeError('rocprofv3 not found')
    child = [sys.executable, os.path.join(ROOT, 'bench.py'), '--steps', '2', '--warmup', '1', '--no-cpu-baseline',
             '--no-kernel-timing', '--no-traffic', '--config', args.config, '--batch', str(batch), '--size', str(size)]
    if args.math:
        child += ['--math', args.math]
    if args.storage:
        child += ['--storage', args.storage]
    if int(args.tune, 0):
        child += ['--tune', args.tune]
    steps = 3
    tot = {}
    tmp = tempfile.mkdtemp(prefix='scd_pmc_', dir='/tmp')
    env = dict(os.environ, TMPDIR='/tmp')
    try:
        for counter in ('FETCH_SIZE', 'WRITE_SIZE'):
            d = os.path.join(tmp, counter)
            subprocess.run([prof, '--pmc', counter, '--output-format', 'csv', '-d', d, '-o', 'run', '--', *child],
                           cwd='/tmp', env=env, timeout=timeout_s, check=True, stdout=subprocess.DEVNULL,
                           stderr=subprocess.DEVNULL)
            found = [os.path.join(dp, f) for dp, _, fs in os.walk(d) for f in fs if f.endswith('counter_collection.csv')]
            if not found:
                raise RuntimeError(f'{counter}: no counter_collection.csv')
            fam = {'igemm': 0.0, 'wgrad': 0.0, 'other': 0.0, 'torch': 0.0}
            with open(found[0]) as f:
                for r in csv.DictReader(f):
                    if r['Counter_Name'] == counter:
                        fam[_conv_family(r['Kernel_Name'])] += float(r['Counter_Value'])
            tot[counter] = fam
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    by = {k: (2.0 * tot['FETCH_SIZE'][k] + tot['WRITE_SIZE'][k]) * 1024.0 / steps for k in tot['FETCH_SIZE']}
    conv = ('igemm', 'wgrad')
    return {"bytes_per_step": round(sum(by[k] for k in conv)), "by_family": {k: round(v) for k, v in by.items()},
            "fetch_bytes_per_step": round(2.0 * sum(tot['FETCH_SIZE'][k] for k in conv) * 1024.0 / steps),
            "write_bytes_per_step": round(sum(tot['WRITE_SIZE'][k] for k in conv) * 1024.0 / steps),
            "source": "measured by this run: two child processes of this workload (3 steps each) under rocprofv3 "
                      "--pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), FETCH x2 (gfx950 wide-read correction), "
                      "KiB x 1024 / 3 steps; L2-miss fabric bytes of the igemm / wgrad kernels (bytes_per_step; "
                      "by_family adds libscd's non-conv kernels ('other') and torch's ('torch': AdamW); Infinity-Cache hits "
                      "included, MI355X_MICROARCH.md HBM)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=5)
    ap.add_argument('--config', default='baseline_siamese')
    ap.add_argument('--batch', type=int, default=None, help='per-GPU batch (default: config TRAINER.BATCH_SIZE)')
    ap.add_argument('--size', type=int, default=None)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-kernel-timing', action='store_true')
    ap.add_argument('--no-traffic', action='store_true',
                    help='skip the live PMC traffic passes (two rocprofv3 child runs of this workload)')
    ap.add_argument('--math', default=None, choices=['f32', 'x3', 'x5', 'bf16', 'h2'],
                    help='conv arithmetic (default: from the config, engine.conv_math_for: MODEL.PRECISION fp32 -> h2)')
    ap.add_argument('--tune', default='0', help='process-default SCD_TUNE_* bits (hex or decimal; A/B of kernel variants)')
    ap.add_argument('--storage', default=None, choices=['fp32', 'bf16'],
                    help='activation / gradient storage (default: engine.act_storage_for: bf16 for the bf16 arithmetic)')
    args = ap.parse_args()

    rank, local_rank, world = parallel.init_distributed()
    dev = torch.device('cuda', parallel.device_index(local_rank))
    torch.cuda.set_device(dev)
    hip.load_library()
    if int(args.tune, 0):
        hip.set_tune(int(args.tune, 0))

    cfg = experiment_manager.load_cfg(args.config)
    if args.math:
        cfg.MODEL.CONV_MATH = args.math
    if args.storage:
        cfg.MODEL.ACT_STORAGE = args.storage
    math = engine.conv_math_for(cfg)  # create_network gives the model this arithmetic (hip.conv_scope per forward)
    storage = 'bf16' if engine.act_storage_for(cfg, math) == torch.bfloat16 else 'fp32'  # activations in HBM
    dtype = {'bf16': 'bf16', 'h2': 'f32 (h2 split-fp16)', 'x3': 'f32 (x3 split-bf16)',
             'x5': 'f32 (x5 split-bf16, 5 products)', 'f32': 'f32'}[math]
    batch = args.batch or int(cfg.TRAINER.BATCH_SIZE)
    size = args.size or int(cfg.AUGMENTATION.CROP_SIZE)
    torch.manual_seed(cfg.SEED)
    net = networks.create_network(cfg).to(dev)
    net = parallel.wrap_ddp(net, dev)
    net.train()
    try:
        opt = torch.optim.AdamW(net.parameters(), lr=float(cfg.TRAINER.LR), weight_decay=0.01, fused=True)
    except (RuntimeError, TypeError):
        opt = torch.optim.AdamW(net.parameters(), lr=float(cfg.TRAINER.LR), weight_decay=0.01)
    gen = torch.Generator(device=dev).manual_seed(parallel.rank_seed(cfg.SEED, rank))
    b = datasets.synthetic_batch(cfg, batch, dev, gen, size)
    hip.ensure_device(b['x_t1'])

    def step():
        opt.zero_grad(set_to_none=True)
        loss = trainers.step_loss(cfg, net(b['x_t1'], b['x_t2']), b, net)  # the config's trainer recipe
        loss.backward()
        opt.step()
        return loss

    for _ in range(args.warmup):
        loss = step()
    torch.cuda.synchronize()
    first_loss = float(loss.item())

    parallel.barrier(dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    parallel.barrier(dev)
    dt_local = time.perf_counter() - t0
    dt = parallel.allreduce_max(dt_local, dev)
    last_loss = float(loss.item())

    value = batch * world * args.steps / dt
    ms = 1000.0 * dt / args.steps
    f3, fT = conv_flops(cfg, batch, size)
    result = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "image-pairs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": dtype,
        "data": "synthetic (on-device U[0,1) pairs, Bernoulli(0.05) change masks; random-init weights)",
        "config": {"workload": f"{args.config}: {cfg.MODEL.TYPE} TOPOLOGY {list(cfg.MODEL.TOPOLOGY)}, "
                               f"{cfg.MODEL.IN_CHANNELS}-ch SAR+optical, {size}x{size}, bs={batch}/GPU, "
                               f"conv math {math}, {storage} activation storage, train step incl. AdamW",
                   "global_batch": batch * world, "tile": size, "parallelism": f"dp{world}",
                   "topology": list(cfg.MODEL.TOPOLOGY)},
        "loss_first_last": [round(first_loss, 6), round(last_loss, 6)],
    }
    if cfg.MODEL.TYPE == 'siameseunet':  # SURVEY 8(d) formula (273.3 GF/pair at 256^2, 5-ch)
        dpeak = PEAKS[math]
        per_gpu = f3 / batch * (value / world)
        result["step_roofline"] = {
            "formula": f"3x3-stack train FLOP/pair x pairs/s/GPU / the {math} arithmetic's matrix-core peak "
                       f"({dpeak:.1f} TFLOP/s)",
            "gflop_per_pair_3x3": round(f3 / batch / 1e9, 2),
            "frac": round(per_gpu / (dpeak * 1e12), 4),
            "nominal_frac_of_fp32_mfma_peak": round(per_gpu / (FP32_MFMA_PEAK_TFLOPS * 1e12), 4)}

    if not args.no_kernel_timing:
        # every rank runs the instrumented steps (DDP's collectives must match); rank 0 records the HIP events
        reps = 2
        timer = KernelTimer() if rank == 0 else None
        if timer is not None:
            timer.install()
            timer.active = True
        for _ in range(reps):
            step()
        torch.cuda.synchronize()
        parallel.barrier(dev)
    if rank == 0 and not args.no_kernel_timing:
        timer.active = False
        summ = timer.summary()
        t_ms = sum(t for _, t in summ.values()) / reps
        # algorithmic conv FLOPs for the Siamese U-Net; other models: the launched conv FLOPs
        flop_step = f3 + fT if cfg.MODEL.TYPE == 'siameseunet' else timer.launched_flops(reps)
        achieved = flop_step / (t_ms * 1e-3) / 1e12
        traffic = None
        if world == 1 and not args.no_traffic:
            try:
                traffic = live_traffic(args, batch, size)
            except Exception as e:  # noqa: BLE001 - reported in the line, never fatal to the bench
                traffic = {"bytes_per_step": None, "source": f"live PMC passes failed: {type(e).__name__}: {e}"}
            alg = timer.alg_bytes(reps)
            traffic["algorithmic_bytes_per_step"] = round(alg)
            if traffic.get("bytes_per_step"):
                traffic["traffic_over_algorithmic"] = round(traffic["bytes_per_step"] / alg, 3)
            other = (traffic.get("by_family") or {}).get("other")
            if other:
                # the non-conv libscd kernels (HBM-bound by design): their bytes over the step time no conv kernel
                # covers (the step has no idle between launches, profiles/r05_step_timeline.txt), an upper bound on
                # their time, so a lower bound on their rate
                rest_ms = ms - t_ms
                traffic["other_family"] = {
                    "bytes_per_step": round(other), "non_conv_ms_per_step": round(rest_ms, 3),
                    "tb_per_s": round(other / (rest_ms * 1e-3) / 1e12, 3) if rest_ms > 0 else None,
                    "peak_tb_per_s": HBM_PEAK_TBS}
        peak, shares = timer.peak()
        result["roofline"] = {
            "bound": "mfma", "achieved": round(achieved, 2), "peak": round(peak, 1), "unit": "TFLOP/s",
            "frac": round(achieved / peak, 4), "traffic": traffic,
            "peak_basis": f"conv math {math}: share of executed conv FLOPs per arithmetic {shares} (peaks: x3 "
                          f"{X3_PEAK_TFLOPS:.1f} = bf16 dense {BF16_MFMA_PEAK_TFLOPS:.1f} / 6 products, h2 "
                          f"{H2_PEAK_TFLOPS:.1f} = fp16 dense / 3 products, bf16 {BF16_MFMA_PEAK_TFLOPS:.1f}, fp32 MFMA "
                          f"{FP32_MFMA_PEAK_TFLOPS}); combined flop-weighted harmonically",
            "frac_of_fp32_mfma_peak": round(achieved / FP32_MFMA_PEAK_TFLOPS, 4),
            "kernel": "igemm + wgrad (all conv launches of one training step: 3x3 fwd/dgrad/wgrad, "
                      "ConvT fwd/dgrad/wgrad)",
            "flop_per_step": flop_step,
            "kernel_ms_per_step": round(t_ms, 3),
            "launches_per_step": {k: v[0] // reps for k, v in summ.items()},
            "ms_per_family": {k: round(v[1] / reps, 3) for k, v in summ.items()},
        }
        # the same HIP events per kernel class; the class with the most time is the step's dominant kernel
        classes = timer.by_class(reps)
        result["roofline"]["by_class"] = classes
        if classes:
            dom = max(classes, key=lambda k: classes[k]["ms_per_step"])
            result["roofline"]["dominant_kernel"] = dict(classes[dom], **{"class": dom})
    if parallel.is_distributed():  # every rank: the probe steps and the report run collectives
        probe = parallel.ExposedAllreduceProbe(net.module, dev)
        exposed = []
        for _ in range(3):
            opt.zero_grad(set_to_none=True)
            loss = trainers.step_loss(cfg, net(b['x_t1'], b['x_t2']), b, net)
            probe.begin()
            loss.backward()
            exposed.append(probe.end())
            opt.step()
        probe.remove()
        rep = parallel.distributed_report(1000.0 * dt_local / args.steps, exposed, dev)
        rep['bucket_cap_mb'] = 16
        result["distributed"] = rep
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(cfg, size=size)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if parallel.is_distributed():
        torch.distributed.destroy_process_group()


if __name__ == '__main__':
    main()
