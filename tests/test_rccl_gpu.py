"""RCCL on one MI355X: a one-rank "nccl" (= librccl) process group carrying the data-parallel path.

The multi-rank tests rehearse two ranks on one GPU over gloo (RCCL refuses two ranks on one device); this one runs the
collectives themselves on RCCL: device all-reduces and the barrier, then a training step through DDP's RCCL gradient
buckets (16 MB buckets, sum hook of the exact-DataParallel mode) whose gradients must equal the same step without DDP
bit for bit (a sum over one rank is the identity).
"""
import os
import socket
import tempfile

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _worker(rank, port, out_dir):
    os.environ.update(RANK='0', LOCAL_RANK='0', WORLD_SIZE='1', MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    import torch.distributed as dist
    from multimodal_siamese_cd_amd import hip, parallel, trainers
    from multimodal_siamese_cd_amd.utils import networks
    from oracle.golden import Fixture
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    dist.init_process_group('nccl', rank=0, world_size=1, device_id=dev)
    out = {'backend': dist.get_backend()}
    t = torch.arange(1 << 20, device=dev, dtype=torch.float32)
    ref = t.clone()
    dist.all_reduce(t)
    dist.barrier(device_ids=[0])
    torch.cuda.synchronize()
    out['allreduce_identity'] = bool(torch.equal(t, ref))
    hip.load_library()
    fx = Fixture('siamese_t32-64')
    cfg = fx.package_cfg()
    b = {k: v.to(dev) for k, v in fx.batch().items()}
    grads = []
    for use_ddp in (False, True):
        net = networks.create_network(cfg)
        with torch.no_grad():
            for k, p in net.module.named_parameters():
                p.copy_(torch.from_numpy(fx.params0[k]))
        net = net.to(dev).train()
        if use_ddp:
            net = parallel.wrap_ddp(net, dev, exact_dataparallel=True, single_rank=True)
            out['wrapped'] = type(net).__name__
        y = net(b['x_t1'], b['x_t2'])
        loss = trainers.step_loss(cfg, y, b, net)
        loss.backward()
        torch.cuda.synchronize()
        mod = net.module
        grads.append({n: p.grad.detach().cpu() for n, p in mod.named_parameters() if p.grad is not None})
        out[f'loss_{int(use_ddp)}'] = loss.item()
    out['same_grads'] = sorted(grads[0]) == sorted(grads[1]) and all(torch.equal(grads[0][n], grads[1][n])
                                                                    for n in grads[0])
    out['n_grads'] = len(grads[0])
    torch.save(out, os.path.join(out_dir, 'rccl.pt'))
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_rccl_one_rank_collectives_and_ddp_buckets():
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(_free_port(), d), nprocs=1, join=True)
        out = torch.load(os.path.join(d, 'rccl.pt'), weights_only=True)
    assert out['backend'] == 'nccl'
    assert out['allreduce_identity']
    assert out['wrapped'] == 'DistributedDataParallel'
    assert out['loss_0'] == out['loss_1']
    assert out['n_grads'] > 0 and out['same_grads']
