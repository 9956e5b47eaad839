"""Multi-process (world_size 2, gloo, CPU) checks of the data-parallel plumbing the
benchmark and the evaluation use: group sharding, max-over-ranks timing, MPJPE
reduction.  The GPU path uses the same functions over RCCL."""
import os
import socket

import numpy as np
import torch
import torch.multiprocessing as mp

from posu import dist as pdist


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    r, _, w = pdist.init('gloo')
    assert (r, w) == (rank, world)
    mine = pdist.shard_groups(10, r, w)
    # per-rank wall time: the job time is the slowest rank's
    tmax = pdist.max_over_ranks(1.0 + r)
    # MPJPE over all groups = (sum of per-rank error sums) / (sum of counts)
    rng = np.random.default_rng(0)
    errs = rng.uniform(0, 100, size=(10, 16))
    local = errs[mine]
    s, c = pdist.sum_over_ranks([local.sum(), local.size])
    out[rank] = (mine, tmax, s / c, pdist.throughput(128, 20, w, tmax))
    torch.distributed.destroy_process_group()


def test_two_rank_sharding_timing_and_mpjpe():
    world = 2
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
        res = dict(out)
    shards = [res[r][0] for r in range(world)]
    assert sorted(sum(shards, [])) == list(range(10))
    assert not set(shards[0]) & set(shards[1])
    assert res[0][1] == res[1][1] == 2.0
    ref = np.random.default_rng(0).uniform(0, 100, size=(10, 16)).mean()
    np.testing.assert_allclose(res[0][2], ref, rtol=1e-12)
    np.testing.assert_allclose(res[1][2], ref, rtol=1e-12)
    assert res[0][3] == 2 * 128 * 20 / 2.0


def test_bench_launcher_starts_one_rank_per_gpu_dry_run():
    """`python bench.py --gpus 2` starts its own two ranks (torch.distributed.run, before any
    GPU call) and the rank code checks the world size: the same launcher and rank path the
    driver's 1->8 GPU scaling run takes, here with gloo and no GPU work (--dry-run)."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, OMP_NUM_THREADS='1')
    env.pop('WORLD_SIZE', None)
    out = subprocess.run([sys.executable, os.path.join(repo, 'bench.py'), '--gpus', '2', '--dry-run', '--steps', '3',
                          '--warmup', '1', '--groups', '5'], capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, out.stdout  # rank 0 prints one line
    d = json.loads(lines[0])
    assert d['n_gpus'] == 2 and d['dry_run']
    assert d['per_rank_frames'] == [4 * 5 * 3, 4 * 5 * 3]
    # a rank launched with a WORLD_SIZE that disagrees with --gpus refuses to run
    bad = subprocess.run([sys.executable, os.path.join(repo, 'bench.py'), '--gpus', '2', '--dry-run'],
                         capture_output=True, text=True, timeout=120,
                         env=dict(env, WORLD_SIZE='1', RANK='0', LOCAL_RANK='0'))
    assert bad.returncode != 0 and 'WORLD_SIZE=1 but --gpus 2' in bad.stderr


# ---------------------------------------------------------------- staged training backward
class _FakeStagePlan:
    """The stage interface of posu.train_plan.TrainPlan on CPU tensors (stage i: y = x @ W_i,
    stage 4 also returns its input as the 'deconv features'), logging when each stage's
    gradients are computed -- to test the autograd / DDP structure without a GPU."""
    NSTAGES = 5

    def __init__(self, weights, log):
        self.w, self.log = weights, log

    def stage_params(self, i):
        return [self.w[i]]

    def forward_stage(self, i, x, nseg):
        with torch.no_grad():
            if i == 0:
                x = torch.cat(x, 0)
            y = x @ self.w[i]
        return ((y, x) if i == 4 else y), x

    def backward_stage(self, i, x, gouts, nseg):
        from posu.train_plan import _Grads
        g = gouts[0]
        if i == 4 and gouts[1] is not None:
            pass   # the features' gradient enters below through gx
        grads = _Grads(None)
        self.log.append(('grad', i))
        grads[self.w[i]] = torch.einsum('nhwc,nhwd->cd', x, g)
        gx = g @ self.w[i].t()
        if i == 4 and gouts[1] is not None:
            gx = gx + gouts[1]
        return (None if i == 0 else gx), grads.close()


class _FakeNet(torch.nn.Module):
    def __init__(self, log, seed):
        super().__init__()
        g = torch.Generator().manual_seed(seed)
        self.w = torch.nn.ParameterList([torch.nn.Parameter(torch.randn(600, 600, generator=g) * 0.04) for _ in range(5)])
        self.plan = _FakeStagePlan(self.w, log)

    def forward(self, views):
        from posu.train_plan import train_forward
        return train_forward(self, self.plan, views, len(views))


def _ddp_worker(rank, world, port, out):
    import torch.distributed as dist
    from posu import train_plan
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    g = torch.Generator().manual_seed(100 + rank)
    views = [torch.randn(2, 3, 1, 600, generator=g) for _ in range(4)]   # 1.4 MB per stage: one bucket each
    res = {}
    for mode in ('delayed', 'joined'):
        train_plan.GRAD_HANDOFF = mode
        log = []
        local = _FakeNet([], 5)
        hm, x1, f = local(views)
        (hm.square().sum() + 0.5 * x1.sum() + 0.25 * f.square().sum()).backward()
        local_grads = torch.cat([p.grad.flatten() for p in local.parameters()])
        # autograd reference: the same math without the stage Functions
        ref = _FakeNet([], 5)
        y = torch.cat(views, 0)
        ys = []
        for w in ref.w:
            y = y @ w
            ys.append(y)
        (ys[4].square().sum() + 0.5 * ys[0].sum() + 0.25 * ys[3].square().sum()).backward()
        ref_grads = torch.cat([p.grad.flatten() for p in ref.parameters()])

        net = _FakeNet(log, 5)
        ddp = torch.nn.parallel.DistributedDataParallel(net, bucket_cap_mb=1e-4)

        def hook(state, bucket):
            log.append(('allreduce', bucket.index()))
            fut = dist.all_reduce(bucket.buffer(), async_op=True).get_future()
            return fut.then(lambda f: f.value()[0] / world)
        ddp.register_comm_hook(None, hook)
        for _ in range(2):   # DDP builds its per-stage buckets from the first iteration's order
            log.clear()
            net.zero_grad(set_to_none=True)
            hm, x1, f = ddp(views)
            (hm.square().sum() + 0.5 * x1.sum() + 0.25 * f.square().sum()).backward()
        ddp_grads = torch.cat([p.grad.flatten() for p in net.parameters()])
        gathered = [torch.empty_like(local_grads) for _ in range(world)]
        dist.all_gather(gathered, local_grads)
        res[mode] = (list(log), float((local_grads - ref_grads).abs().max()),
                     float((ddp_grads - torch.stack(gathered).mean(0)).abs().max()), float(ref_grads.abs().max()))
    out[rank] = res
    dist.destroy_process_group()


def test_staged_backward_overlaps_ddp_allreduce_with_earlier_stages():
    """The training forward is five stage Functions (posu.train_plan._StageFn): DDP's first
    gradient bucket is all-reduced while earlier stages are still in backward -- before the
    stem stage's gradients are computed -- and the gradients equal plain autograd's (local) and
    the mean of the ranks' local gradients (DDP), with the layer1 and deconv features
    differentiable."""
    world = 2
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_ddp_worker, args=(world, port, out), nprocs=world, join=True)
        res = dict(out)
    for r in range(world):
        for mode, (log, err_local, err_ddp, scale) in res[r].items():
            assert err_local <= 1e-5 * scale, (mode, err_local)
            assert err_ddp <= 1e-5 * scale, (mode, err_ddp)
            grads = [e for e in log if e[0] == 'grad']
            assert [e[1] for e in grads] == [4, 3, 2, 1, 0], log
            first_ar = next(k for k, e in enumerate(log) if e[0] == 'allreduce')
            assert first_ar < log.index(('grad', 0)), (mode, log)
            if mode == 'joined':   # stage 4's bucket goes out before stage 3's backward starts
                assert first_ar < log.index(('grad', 3)), log
            else:                  # handed over by stage 3: out before stage 2's backward
                assert first_ar < log.index(('grad', 2)), log
