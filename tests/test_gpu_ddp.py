"""Data-parallel training (BASELINE configs[3]) through torch DistributedDataParallel
over the HIP training path: two ranks on the box's one GPU (gloo carries the
all-reduce here; the 8-GPU bench uses RCCL, same DDP code).  After backward every
rank must hold the mean of the ranks' local gradients, with per-rank (per-view)
BatchNorm statistics as in the reference (no SyncBN, train.py:223)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(repo, 'pose-unsupervised_amd', 'lib'), repo]
    import torch.distributed as dist
    from core.loss import JointsMSELoss
    from models.multiview_pose_resnet import get_multiview_pose_net
    from models.pose_resnet import get_pose_net
    from posu import synthetic as syn
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    dev = torch.device('cuda', 0)
    cfg = syn.make_cfg(num_layers=18, image_size=64)

    def make():
        net = get_pose_net(cfg, is_train=False, precision='fp32')
        net.load_state_dict(syn.synthetic_state_dict(net.state_dict(), seed=3))
        return net.to(dev).train()

    views = [v.to(dev) for v in syn.synthetic_views(4, 2, 64, seed=60 + rank)]   # this rank's shard
    tgt = torch.rand(4, 2, 16, 16, 16, generator=torch.Generator().manual_seed(70 + rank)).to(dev)
    w = torch.ones(2, 16, 1, device=dev)
    crit = JointsMSELoss(use_target_weight=True)

    def loss_of(model):
        out, _, _, _ = model(views)
        return sum(crit(o, tgt[v], w) for v, o in enumerate(out))

    local = make()
    loss_of(get_multiview_pose_net(local, cfg)).backward()
    local_grads = torch.cat([p.grad.flatten() for p in local.parameters()])

    net = make()
    ddp = torch.nn.parallel.DistributedDataParallel(get_multiview_pose_net(net, cfg), bucket_cap_mb=4)
    loss_of(ddp).backward()
    ddp_grads = torch.cat([p.grad.flatten() for p in net.parameters()])
    gathered = [torch.empty_like(local_grads) for _ in range(world)]
    dist.all_gather(gathered, local_grads)
    mean = torch.stack(gathered).mean(0)
    out[rank] = (float((ddp_grads - mean).abs().max()), float(mean.abs().max()),
                 float((gathered[0] - gathered[1]).abs().max()))
    dist.destroy_process_group()


def test_ddp_gradients_are_the_mean_of_the_ranks_local_gradients(cuda):
    world = 2
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
        res = dict(out)
    for r in range(world):
        err, scale, spread = res[r]
        assert spread > 1e-3 * scale          # the shards really differ
        assert err <= 1e-5 * scale + 1e-7, res
