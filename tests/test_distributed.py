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
