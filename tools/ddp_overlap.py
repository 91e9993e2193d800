"""DDP gradient-bucket timing of the bench step: when each bucket's all-reduce can start, relative to the backward.

    SCD_DIST_BACKEND=gloo SCD_RANKS_SHARE_GPU=1 torchrun --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29511 tools/ddp_overlap.py [--batch 8] [--config baseline_siamese]

A communication hook wraps DDP's all-reduce: when DDP hands it a bucket (all its gradients produced) it records a
CUDA event on the backward's stream -- the GPU time from which RCCL's all-reduce of that bucket can run -- and the
host time of the call.  Rank 0 prints one JSON object: per bucket its size, the model parts it holds, the GPU ready
time and the host call time in ms after the backward started, and the backward's GPU end; `ready_before_end_ms` is
how much of the backward is still to run when the bucket becomes ready (the overlap window of its all-reduce).
On this one-GPU rehearsal gloo carries the all-reduce (a host copy); the timing of the buckets is the engine's.
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from multimodal_siamese_cd_amd import hip, parallel, trainers  # noqa: E402
from multimodal_siamese_cd_amd.utils import datasets, experiment_manager, networks  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='baseline_siamese')
    ap.add_argument('--batch', type=int, default=8)
    ap.add_argument('--size', type=int, default=256)
    ap.add_argument('--steps', type=int, default=3)
    args = ap.parse_args()
    rank, local_rank, world = parallel.init_distributed()
    dev = torch.device('cuda', parallel.device_index(local_rank))
    torch.cuda.set_device(dev)
    hip.load_library()
    cfg = experiment_manager.load_cfg(args.config)
    torch.manual_seed(0)
    net = networks.create_network(cfg).to(dev).train()
    net = parallel.wrap_ddp(net, dev)
    names = {id(p): n for n, p in net.module.named_parameters()}
    log = []

    def hook(state, bucket):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        parts = sorted({names[id(p)].split('.')[0] + ('.' + names[id(p)].split('.')[2]
                                                      if names[id(p)].startswith(('encoder.', 'decoder.')) else '')
                        for p in bucket.parameters()})
        log.append(dict(index=bucket.index(), mb=bucket.buffer().numel() * 4 / 2 ** 20, parts=parts, ev=ev,
                        host=time.perf_counter()))
        buf = bucket.buffer()
        buf.div_(dist.get_world_size())
        fut = dist.all_reduce(buf, async_op=True).get_future()
        return fut.then(lambda f: f.value()[0])

    if parallel.is_distributed():
        net.register_comm_hook(None, hook)
    gen = torch.Generator(device=dev).manual_seed(parallel.rank_seed(1, rank))
    b = datasets.synthetic_batch(cfg, args.batch, dev, gen, args.size)
    result = None
    for it in range(args.steps):
        log.clear()
        net.zero_grad(set_to_none=True)
        loss = trainers.step_loss(cfg, net(b['x_t1'], b['x_t2']), b)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        h0 = time.perf_counter()
        e0.record()
        loss.backward()
        e1.record()
        torch.cuda.synchronize()
        end = e0.elapsed_time(e1)
        rows = [dict(index=r['index'], mb=round(r['mb'], 2), parts=r['parts'],
                     gpu_ready_ms=round(e0.elapsed_time(r['ev']), 3), host_call_ms=round((r['host'] - h0) * 1e3, 3),
                     ready_before_end_ms=round(end - e0.elapsed_time(r['ev']), 3)) for r in log]
        result = dict(config=args.config, batch_per_rank=args.batch, world=world,
                      backend=dist.get_backend() if parallel.is_distributed() else None,
                      backward_gpu_ms=round(end, 3), buckets=rows)
    if rank == 0:
        print(json.dumps(result, indent=1))
    if parallel.is_distributed():
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
