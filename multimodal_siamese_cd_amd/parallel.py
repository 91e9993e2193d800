"""One process per GPU data parallelism over RCCL (torch.distributed backend "nccl" = librccl on ROCm).

Replaces the reference's single-process `nn.DataParallel(model)` (utils/networks.py:27).  Each rank owns a
full replica and its own shard of image pairs (independent synthetic generator seeded per rank); the only
data-path collective is the gradient all-reduce that DistributedDataParallel buckets and launches as the
stage Functions (one per encoder level, then the decoder) return their gradients.  BatchNorm statistics stay per rank (like DataParallel's
per-replica statistics) and running statistics are broadcast from rank 0 each forward
(`broadcast_buffers=True`, DataParallel's replica-0 semantics, torch/nn/parallel/data_parallel.py:88-90).
"""
from __future__ import annotations

import contextlib
import os

import torch
import torch.distributed as dist


def env_rank():
    return int(os.environ.get('RANK', 0)), int(os.environ.get('LOCAL_RANK', 0)), int(os.environ.get('WORLD_SIZE', 1))


def device_index(local_rank: int) -> int:
    """The GPU of a rank: its local rank (one process per GPU).  SCD_RANKS_SHARE_GPU=1 folds ranks onto the
    visible devices (a rehearsal of the multi-rank path on a one-GPU machine, with SCD_DIST_BACKEND=gloo)."""
    if os.environ.get('SCD_RANKS_SHARE_GPU') == '1':
        return local_rank % max(torch.cuda.device_count(), 1)
    return local_rank


def init_distributed(backend: str | None = None):
    """Initialise the process group from torchrun's env; returns (rank, local_rank, world_size)."""
    rank, local_rank, world = env_rank()
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = os.environ.get('SCD_DIST_BACKEND') or ('nccl' if torch.cuda.is_available() else 'gloo')
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        if backend == 'nccl':
            torch.cuda.set_device(device_index(local_rank))
            dist.init_process_group(backend, device_id=torch.device('cuda', device_index(local_rank)))
        else:
            dist.init_process_group(backend)
    return rank, local_rank, world


def is_distributed() -> bool:
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def rank_seed(seed: int, rank: int) -> int:
    """Independent per-rank data stream (weak scaling: each rank draws its own pairs)."""
    return int(seed) * 1_000_003 + 7919 * int(rank)


def params_outside_forward(module) -> tuple:
    """Names of submodules whose parameters a model holds but never uses in forward.

    The reference keeps such modules for state_dict compatibility, e.g. DualTaskSiameseUNet.outc_sem_change
    (utils/networks.py:174): it never receives a gradient.  Models declare them in `PARAMS_OUTSIDE_FORWARD`.
    """
    return tuple(getattr(module, 'PARAMS_OUTSIDE_FORWARD', ()))


def allreduce_sum_(t: torch.Tensor, group=None) -> torch.Tensor:
    """In-place SUM over the ranks (the exact-DataParallel loss sums)."""
    if is_distributed():
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t


def sum_allreduce_hook(process_group, bucket):
    """DDP communication hook: gradient buckets SUMMED over the ranks (DDP's default divides by the world size).
    With one global loss per step (exact-DataParallel mode) each rank's gradient is its shard's part of the global
    gradient, and nn.DataParallel reduce-adds the replicas' gradients (torch/nn/parallel/data_parallel.py)."""
    group = process_group if process_group is not None else dist.group.WORLD
    fut = dist.all_reduce(bucket.buffer(), group=group, async_op=True).get_future()
    return fut.then(lambda f: f.value()[0])


def global_sums(local: torch.Tensor) -> torch.Tensor:
    """The SUM over ranks of `local`, differentiable with the identity gradient to `local` (d global / d local = 1
    per rank): the torch form of the exact-DataParallel loss sums, for losses written in torch (tests, oracle)."""
    if not is_distributed():
        return local
    tot = local.detach().clone()
    dist.all_reduce(tot, op=dist.ReduceOp.SUM)
    return local + (tot - local.detach())


def wrap_ddp(wrapper, device=None, bucket_cap_mb: int = 16, find_unused_parameters: bool | None = None,
             exact_dataparallel: bool = False, single_rank: bool = False):
    """Replace the DataParallel-style wrapper's pass-through by DDP when running under torchrun.

    Keeps the `.module` attribute and `module.` state_dict prefix of the reference's wrapper.

    Overlap.  The encoder runs one autograd Function per level (engine.EncoderLevelFn / SiameseLevelFn), so a level's
    gradients reach DDP when that level's backward returns, deepest level first.  16 MB buckets (SiameseUNet: 59 MB
    of fp32 gradients, the decoder's 21 MB ready together, then down4 19 MB, down3 14 MB, ...) let the all-reduce of
    each bucket run on RCCL's stream while the shallower, costlier levels' backward continues; only the last bucket
    (the shallow levels, < 4 MB) is exposed.
    Parameters a model declares outside its forward graph (`params_outside_forward`, e.g. the dual-task model's
    outc_sem_change) are excluded from DDP (never bucketed, never reduced: they never get a gradient), so the default
    `find_unused_parameters=None` runs without DDP's per-step unused-parameter search; without the exclusion, the
    bucket holding such a parameter would never be reduced and the next step would raise.  (Until round 6 the search
    was turned on for such models instead; with it dtsiamese's last bucket, ready 5 ms before the backward's end,
    measured 17.9 MB: profiles/r06_rehearsal_2rank/.)

    Loss semantics.  Default (the throughput mode): every rank takes power_jaccard_loss over its own shard and DDP
    averages the gradients, i.e. the gradient of the MEAN of the per-shard losses.  The reference's nn.DataParallel
    takes ONE loss over the gathered batch (utils/networks.py:27, train_supervised.py:75), a different function of
    the logits (Jaccard is a ratio of batch sums: 7e-6 apart at bs=2).  exact_dataparallel=True reproduces
    it: the loss kernels' partial sums (I, sum p^2 + t^2 per term) are SUM-all-reduced before the loss is formed
    (three floats per term), and the gradient buckets are SUMMED (sum_allreduce_hook).  The loss reduction belongs
    to the wrapped model, not to the process: the wrapper is marked (`exact_dataparallel`), and only a loss formed
    under `loss_scope(net)` (trainers.step_loss(cfg, out, batch, net)) runs the collective.
    BatchNorm statistics stay per rank and running statistics come from rank 0 (broadcast_buffers) in both modes,
    as DataParallel's per-replica statistics with replica 0's buffers.
    `single_rank`: wrap even in a one-rank process group (the RCCL / DDP bucket path on one GPU,
    tests/test_rccl_gpu.py); without it a single process keeps the reference's pass-through wrapper.
    """
    if not is_distributed() and not (single_rank and dist.is_available() and dist.is_initialized()):
        return wrapper
    module = wrapper.module if hasattr(wrapper, 'module') else wrapper
    if find_unused_parameters is None:
        # parameters the model declares outside its forward (never a gradient) are left out of DDP's buckets, so no
        # per-step unused-parameter search runs and the gradient buckets follow the readiness order of the others
        outside = params_outside_forward(module)
        ignore = [n for n, _ in module.named_parameters() if n.split('.')[0] in outside]
        if ignore:
            torch.nn.parallel.DistributedDataParallel._set_params_and_buffers_to_ignore_for_model(module, ignore)
        find_unused_parameters = False
    ids = [device.index] if (device is not None and device.type == 'cuda') else None
    ddp = torch.nn.parallel.DistributedDataParallel(module, device_ids=ids, broadcast_buffers=True,
                                                    bucket_cap_mb=bucket_cap_mb, gradient_as_bucket_view=True,
                                                    find_unused_parameters=find_unused_parameters)
    ddp.exact_dataparallel = bool(exact_dataparallel)
    if exact_dataparallel:
        ddp.register_comm_hook(None, sum_allreduce_hook)
    return ddp


def loss_scope(net):
    """The context a training step's loss is formed in: for a model wrapped with exact_dataparallel=True the loss
    kernels' partial sums are SUM-all-reduced over the ranks (engine.loss_reduction); otherwise nothing changes."""
    from . import engine
    if getattr(net, 'exact_dataparallel', False):
        return engine.loss_reduction(allreduce_sum_)
    return contextlib.nullcontext()


def allreduce_max(value: float, device) -> float:
    if not is_distributed():
        return value
    if dist.get_backend() == 'nccl':
        if device is None or getattr(device, 'type', 'cpu') != 'cuda':
            device = torch.device('cuda', torch.cuda.current_device())
    else:
        device = 'cpu'
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def barrier(device=None):
    if is_distributed():
        if device is not None and device.type == 'cuda' and dist.get_backend() == 'nccl':
            dist.barrier(device_ids=[device.index])
        else:
            dist.barrier()


def gather_floats(value: float, device=None) -> list:
    """Every rank's `value`, in rank order (one SUM all-reduce of a one-hot vector)."""
    if not is_distributed():
        return [float(value)]
    if dist.get_backend() == 'nccl':  # RCCL reduces device tensors only
        if device is None or getattr(device, 'type', 'cpu') != 'cuda':
            device = torch.device('cuda', torch.cuda.current_device())
    else:
        device = 'cpu'
    t = torch.zeros(dist.get_world_size(), dtype=torch.float64, device=device)
    t[dist.get_rank()] = float(value)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return [float(v) for v in t.tolist()]


class ExposedAllreduceProbe:
    """The gradient all-reduce time a DDP backward leaves exposed, measured on this rank.

    Every parameter gets a tensor hook that stamps the moment its gradient is produced (a HIP event on the stream
    the backward runs on, or the host clock on CPU); `end()` stamps the return of backward(), by which point DDP's
    reducer has made the compute stream wait for every bucket's all-reduce.  Exposed = end - the last gradient
    stamp: the all-reduce time that overlapped no backward kernel."""

    def __init__(self, module, device=None):
        self.cuda = device is not None and getattr(device, 'type', 'cpu') == 'cuda'
        self.active = False
        self.marks, self.t0, self.t1 = [], None, None
        self.handles = [p.register_hook(self._hook) for p in module.parameters() if p.requires_grad]

    def _stamp(self):
        if self.cuda:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            return e
        import time
        return time.perf_counter()

    def _hook(self, grad):
        if self.active:
            self.marks.append(self._stamp())

    def begin(self):
        self.marks = []
        self.active = True
        self.t0 = self._stamp()

    def end(self) -> dict:
        """{backward_ms, last_grad_ms, exposed_ms} of the backward between begin() and now."""
        self.t1 = self._stamp()
        self.active = False
        if self.cuda:
            torch.cuda.synchronize()
            last = max((self.t0.elapsed_time(m) for m in self.marks), default=0.0)
            total = self.t0.elapsed_time(self.t1)
        else:
            last = max(((m - self.t0) * 1e3 for m in self.marks), default=0.0)
            total = (self.t1 - self.t0) * 1e3
        return {'backward_ms': total, 'last_grad_ms': last, 'exposed_ms': max(total - last, 0.0)}

    def remove(self):
        for h in self.handles:
            h.remove()
        self.handles = []


def distributed_report(ms_per_step: float, exposed: list, device=None) -> dict:
    """The bench line's `distributed` fields (every rank calls it; collectives inside): backend, world size as the
    process group reports it, per-rank ms per step (min / max over ranks), and rank 0's exposed all-reduce
    (median of the probe's steps)."""
    per_rank = gather_floats(ms_per_step, device)
    med = sorted(e['exposed_ms'] for e in exposed)[len(exposed) // 2] if exposed else None
    bwd = sorted(e['backward_ms'] for e in exposed)[len(exposed) // 2] if exposed else None
    return {'backend': dist.get_backend() if is_distributed() else None,
            'world_size': dist.get_world_size() if is_distributed() else 1,
            'ms_per_step_by_rank': {'min': round(min(per_rank), 3), 'max': round(max(per_rank), 3),
                                    'all': [round(v, 3) for v in per_rank]},
            'exposed_allreduce_ms_rank0': None if med is None else round(med, 3),
            'backward_ms_rank0': None if bwd is None else round(bwd, 3),
            'probe_steps': len(exposed)}
