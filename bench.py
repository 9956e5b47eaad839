"""Benchmark of the 4-view hot path (BASELINE.json metric: 4-view 256x256 frames/sec,
fwd + triangulate; MPJPE-mm vs ref).

One step = one batch of 32 groups x 4 views (128 frames, 256x256, synthetic N(0,1)
crops already resident in HBM) through
    PoseResNet-50 forward (bf16 MFMA kernels) -> soft-argmax + crop affine
    -> epipolar loss -> fp64 DLT triangulation,
captured as two hipGraphs per input batch (network | decode+geometry) and replayed.
The timed steps rotate over --batches distinct input batches (3 x 100 MB of crops, more
than the 256 MiB Infinity Cache holds), so no step reads inputs an earlier step left
on-die.

Multi-GPU: `python bench.py --gpus N` starts N ranks itself (one process per GPU,
torch.distributed.run, 127.0.0.1 rendezvous) before this process touches the GPU; the
driver's `python -m torch.distributed.run ... bench.py --gpus N` lands directly in the
rank code.  The global batch of 32 x N groups is sharded over the ranks by
posu.dist.shard_groups (the reference's DistributedSampler order, lib/utils/utils.py:134-141;
every group's crops come from its own generator, so the global batch does not depend on N):
32 groups per rank (weak scaling, no data-path collective), `dist.get_world_size() == N` is
asserted, time = max over ranks, value = all ranks' frames / that time.

Also reported, on the same JSON line (rank 0):
  roofline       -- the network (fused stem + implicit-GEMM MFMA conv stack + fused
                    deconv/head): 14.47 GFLOP/frame x 128 frames per replay / its
                    HIP-event time on the launch stream, against the dense bf16 peak;
  mpjpe_vs_ref_mm -- the bench chain's triangulated joints against the CPU oracle chain
                    (fp32 reference network + soft-argmax + affine + fp64 triangulation)
                    on the same first input batch, as run/test/test_triangulate.py:98-102
                    computes MPJPE (mean / std / max per-joint error, mm);
  triangulation_same_2d_mm_all_ranks -- every rank's device triangulation against the oracle's
                    triangulation of the same device joints, reduced over ranks (posu.dist);
  fp32_mode      -- frames/s of the same pipeline with the exact-f32 kernels;
  parity_mode    -- frames/s of the same pipeline in split fp16 (precision fp16x3: every value a
                    (hi, lo) fp16 pair, hi.hi + lo.hi + hi.lo on the fp16 MFMAs) -- the
                    parity-bearing fast mode: within the BASELINE bars on peaked heatmaps
                    (peaked_parity.fp16x3);
  configs1       -- BASELINE configs[1]: the R50 heatmap forward alone at batch 64, bf16;
  train_mode     -- BASELINE configs[3]: the training step (fwd + bwd + Adam, DDP over RCCL
                    when N > 1), time-bounded (--train-steps);
  cpu_baseline   -- that oracle chain timed on the host cores (rank 0 at N = 1): the full
                    32 x 4 batch (configs[2]) and batch 1 (configs[0]).
`--dry-run` runs the launcher and the rank plumbing on CPU (gloo) without any GPU work.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (os.path.join(REPO, 'pose-unsupervised_amd', 'lib'), REPO):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

GFLOP_PER_FRAME = {(50, 256): 14.47, (152, 384): 76.19, (18, 128): None}
# training step: 3x forward minus the stem's data gradient
TRAIN_GFLOP_PER_FRAME = {(50, 256): 43.1}
PEAK_BF16_TFLOPS = 2500.0
PEAK_F32_TFLOPS = 157.3
METRIC = '4-view 256x256 frames/sec (fwd+triangulate)'
TRAIN_METRIC = '4-view 256x256 training frames/sec (fwd+bwd+Adam, per-view BN)'


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--mode', default='infer', choices=['infer', 'train'],
                    help='infer: BASELINE metric (fwd + triangulate); train: configs[3] training step')
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=5)
    ap.add_argument('--groups', type=int, default=32, help='4-view groups per GPU per step')
    ap.add_argument('--batches', type=int, default=3, help='distinct input batches rotated over the timed steps')
    ap.add_argument('--layers', type=int, default=50)
    ap.add_argument('--size', type=int, default=256)
    ap.add_argument('--precision', default='bf16', choices=['bf16', 'fp16', 'fp32', 'fp16x3'])
    ap.add_argument('--no-graph', action='store_true')
    ap.add_argument('--serial-geo', action='store_true',
                    help='run each batch\'s decode + geometry after its network on one stream (default: on a '
                         'second stream, overlapping the next batch\'s network)')
    ap.add_argument('--adam', default='posu', choices=['posu', 'fused', 'foreach'],
                    help="train mode: posu.optim.Adam (default: posu_adam_step, every parameter in a few "
                         "launches) or torch.optim.Adam's fused kernel / foreach launches")
    ap.add_argument('--no-autotune', action='store_true', help='keep the built-in conv tile heuristic')
    ap.add_argument('--tune-file', default='',
                    help='per-layer tile table: loaded if it exists (no tuning trials run), else written '
                         'after autotuning -- profile runs load it so traces hold no trial launches')
    ap.add_argument('--chunks', type=int, default=None,
                    help='depth-first slices for the HBM-bound stem..layer2 / deconv2..head stages (default: the '
                         'plan\'s per-dtype choice, plan.default_chunks(): 2 for fp16x3, else 1)')
    ap.add_argument('--cpu-baseline-seconds', type=float, default=12.0)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-mpjpe', action='store_true', help='skip the oracle-chain MPJPE check')
    ap.add_argument('--fp32-steps', type=int, default=5, help='timed steps of the exact-f32 mode (0: skip)')
    ap.add_argument('--parity-steps', type=int, default=10,
                    help='timed steps of the split-fp16 parity mode (fp16x3), reported as parity_mode (0: skip)')
    ap.add_argument('--train-steps', type=int, default=10,
                    help='infer mode: timed steps of the configs[3] training step reported as train_mode (0: skip)')
    ap.add_argument('--peaked-steps', type=int, default=1200,
                    help='N = 1: fit steps of the peaked-heatmap network behind mpjpe_vs_ref_mm (0: skip)')
    ap.add_argument('--c1-steps', type=int, default=20,
                    help='infer mode: timed replays of the configs[1] forward (batch 64) reported as configs1 (0: skip)')
    ap.add_argument('--c4-steps', type=int, default=10,
                    help='infer mode: timed steps of configs[4]\'s per-GPU pipeline (R152@384 fp16, 16 groups x 4 '
                         'views) reported as configs4 (0: skip)')
    ap.add_argument('--control-steps', type=int, default=10,
                    help='infer mode: timed steps of the same pipeline with this round\'s plan switches off '
                         '(CONTROL_FLAGS: the previous round\'s plan), reported as control (0: skip)')
    ap.add_argument('--train-last', action='store_true',
                    help='diagnostic: run the training leg after the fp32 / configs1 / control / configs4 legs (the '
                         'round-3 order), optionally with --empty-cache-before-train')
    ap.add_argument('--empty-cache-before-train', action='store_true',
                    help='diagnostic: torch.cuda.empty_cache() before the training leg')
    ap.add_argument('--dry-run', action='store_true', help='launcher + rank plumbing on CPU (gloo), no GPU work')
    ap.add_argument('--train-stream', default='default', choices=['high', 'default'],
                    help='train mode: run the step on a high-priority stream (the weight-gradient side '
                         'stream keeps normal priority, so the data-gradient chain wins dispatch) or on '
                         'the default stream (default; measured equal: 21.82 vs 21.80 ms per step)')
    ap.add_argument('--plan-flag', action='append', default=[], metavar='NAME=VALUE',
                    help='A/B runs: set a boolean (0 / 1) or integer switch of posu.plan / posu.train_plan '
                         '(e.g. S2_CHAIN=0, STEM_CIN_PAD=16) before the plans are built')
    return ap.parse_args()


# the plan switches this round added (posu.plan): off, the plan is the previous round's -- the
# line's `control` legs time it in the same process, so a gain shows on the driver's own box.
# headline (bf16 R50@256): the two-K-group tile 39 among the tuner's candidates again (plan.TILES_KSPLIT,
# back on at the end of round 6: 1 % on the headline and configs[1] with this round's plan); parity_mode (fp16x3): round 6's split streamed tails (layer1-3,
# layer1's down tail, the layers' first conv1 chained), staggered split tiles and the depth-first halves
# (CHUNKS_F16X3 off: whole batches); configs4 (R152@384 fp16):
# round 6's layer1 tails at 96-wide maps.
# (PRECISE_HEAD stays on: it is a precision choice -- +39 us for 2x closer joints -- and the
# control legs compare the plans at the same numerics)
CONTROL_FLAGS = ('TILES_KSPLIT',)
CONTROL_FLAGS_PARITY = ('SPLIT_TAILS', 'TILES_SPLIT_SG', 'CHUNKS_F16X3')   # (SPLIT_TAILS off also drops CHAIN_LAYERS)
CONTROL_FLAGS_C4 = ('TAIL_W96',)


def apply_plan_flags(flags):
    from posu import plan as pl, train_plan as tpl
    for f in flags:
        name, _, val = f.partition('=')
        mod = next((m for m in (pl, tpl) if isinstance(getattr(m, name, None), (bool, int, float))), None)
        if mod is None:
            raise SystemExit('--plan-flag %s: not a switch of posu.plan / posu.train_plan' % f)
        if isinstance(getattr(mod, name), bool):
            if val not in ('0', '1'):
                raise SystemExit('--plan-flag %s: a boolean switch takes 0 or 1' % f)
            setattr(mod, name, val == '1')
        else:
            kind = type(getattr(mod, name))
            try:
                setattr(mod, name, kind(val))
            except ValueError:
                raise SystemExit('--plan-flag %s: a %s switch takes a %s' % (f, kind.__name__, kind.__name__)) from None


# ------------------------------------------------------------------ launcher
def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(args):
    """One process per GPU, started before this process makes any HIP call (the
    reference's mp.spawn + init_process_group, run/pose2d/train.py:129-135)."""
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', str(args.gpus),
           '--master-addr', '127.0.0.1', '--master-port', str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')
    env.setdefault('OMP_NUM_THREADS', '1')
    return subprocess.call(cmd, env=env)


def init_ranks(args, backend, device=None):
    """-> (rank, local, world, dist or None); asserts the job has exactly --gpus ranks."""
    from posu import dist as pdist
    rank, local, world = pdist.env_rank()
    if world != args.gpus:
        raise SystemExit('bench.py: WORLD_SIZE=%d but --gpus %d' % (world, args.gpus))
    dist = None
    if world > 1:
        import torch.distributed as dist
        pdist.init(backend, device=device)
        got = dist.get_world_size()
        assert got == args.gpus, 'process group has %d ranks, expected %d' % (got, args.gpus)
    return rank, local, world, dist


def rank_device(local):
    """(this rank's GPU, process-group backend): cuda:LOCAL_RANK over RCCL ('nccl').  Rehearsal of
    the N-rank path on a box with fewer GPUs (POSU_SHARED_GPU_REHEARSAL=1, never the measured
    line): ranks share the GPUs round-robin and talk over gloo (RCCL refuses two ranks on one GPU)."""
    if os.environ.get('POSU_SHARED_GPU_REHEARSAL') == '1':
        return torch.device('cuda', local % max(1, torch.cuda.device_count())), 'gloo'
    return torch.device('cuda', local), 'nccl'


def gather_per_rank(values, dist, device='cpu'):
    """All ranks' small float vectors (rank order), e.g. [frames, seconds]."""
    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=device)
    if dist is None:
        return [t.tolist()]
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [o.tolist() for o in out]


def dry_run_main(args):
    """The rank plumbing of the real run on CPU (gloo): world size check, per-rank group
    shards, barrier-bracketed timing, max over ranks, all ranks' frames.  No GPU work: the
    per-step work is a stand-in (a small CPU matmul per group), so `value` is not a
    measurement of the hot path and the line says so."""
    from posu import dist as pdist
    rank, local, world, dist = init_ranks(args, 'gloo')
    groups = pdist.shard_groups(args.groups * world, rank, world)
    a = torch.randn(64, 64)

    def step():
        for _ in groups:
            a.mm(a)
    for _ in range(args.warmup):
        step()
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    if dist is not None:
        dist.barrier()
    elapsed = pdist.max_over_ranks(time.perf_counter() - t0)
    per_rank = gather_per_rank([4 * len(groups) * args.steps, elapsed], dist)
    if rank == 0:
        print(json.dumps({'metric': METRIC + ' [dry run: launcher plumbing only, no GPU work]',
                          'value': pdist.throughput(4 * len(groups), args.steps, world, elapsed), 'unit': 'frames/s',
                          'n_gpus': world, 'steps': args.steps, 'warmup': args.warmup, 'dry_run': True,
                          'per_rank_frames': [int(p[0]) for p in per_rank], 'groups_per_rank': len(groups)}))
    if dist is not None:
        dist.destroy_process_group()


# ------------------------------------------------------------------ model / oracle
def build_model(layers, size, precision, device):
    from models.pose_resnet import get_pose_net
    from posu import synthetic as syn
    net = get_pose_net(syn.make_cfg(num_layers=layers, image_size=size), is_train=False, precision=precision)
    net.load_state_dict(syn.synthetic_state_dict(net.state_dict(), seed=syn.calibrated_seed(layers, size),
                                                 bn_stats=syn.load_bn_stats(layers, size)))
    return net.to(device).eval()


def input_views(shard, size, b, device):
    """The 4 views of this rank's groups (`shard`, indices into the global batch) of input
    batch b: every group's crops come from its own generator, so the global batch is the same
    whatever the number of ranks."""
    from posu import synthetic as syn
    return [v.to(device) for v in syn.group_views(4, shard, size, seed=100 + b)]


def pmc_traffic_train(layers, size, precision, groups):
    """HBM bytes of one training step from the newest committed PMC reduction
    (profiles/<round>/pmc_traffic_train.txt, tools/pmc_train_traffic.py), for the default
    training workload; (None, None) otherwise."""
    if (layers, size, precision, groups) != (50, 256, 'bf16', 32):
        return None, None
    import glob
    files = sorted(glob.glob(os.path.join(REPO, 'profiles', 'r*', 'pmc_traffic_train.txt')))
    if not files:
        return None, None
    with open(files[-1]) as f:
        d = json.loads(next(ln for ln in f if ln.startswith('{')))
    return d['traffic_bytes'], {'file': os.path.relpath(files[-1], REPO), 'commit': d.get('commit')}


def pmc_traffic(layers, size, precision, groups):
    """HBM bytes of one network forward from the newest committed PMC reduction
    (profiles/<round>/pmc_traffic_network.txt, written by tools/profile_round.sh with the
    commit it was measured at; the fp16x3 plan's: pmc_traffic_network_fp16x3.txt, round 6), for the
    default workload; (None, None) otherwise."""
    if (layers, size, groups) != (50, 256, 32) or precision not in ('bf16', 'fp16x3'):
        return None, None
    import glob
    name = 'pmc_traffic_network.txt' if precision == 'bf16' else 'pmc_traffic_network_fp16x3.txt'
    files = sorted(glob.glob(os.path.join(REPO, 'profiles', 'r*', name)))
    if not files:
        return None, None
    with open(files[-1]) as f:
        d = json.loads(f.readline())
    return d['traffic_bytes'], {'file': os.path.relpath(files[-1], REPO), 'commit': d.get('commit')}


def oracle_chain(sd, layers, size, views_cpu, host, full=False):
    """CPU oracle of the whole step on one batch: fp32 reference network -> soft-argmax ->
    crop affine -> FundamentalLoss -> fp64 triangulation.  Returns X [G, J, 3] (full: a
    dict with the heatmaps, image-px joints [V, G, J, 2], the loss and X)."""
    from oracle import geometry_ref as G
    from oracle import pose_resnet_ref as PR
    ng = views_cpu[0].shape[0]
    hm, _, _ = PR.pose_resnet_forward(torch.cat(views_cpu, 0), sd, layers)
    sa = G.softargmax2d(hm)
    img = G.transform_back(sa, host['centers'].reshape(-1, 2), host['scales'].reshape(-1, 2), [size // 4] * 2)
    joints = [img[v * ng:(v + 1) * ng] for v in range(4)]
    loss = G.fundamental_loss(joints, [torch.ones(ng, 16, 1)] * 4, host['subjects'], host['F_dict'])
    p2d = torch.stack(joints, 1).reshape(ng * 4, 16, 2).double().numpy()   # group-major, view-minor
    X = G.triangulate_poses(host['cams'], p2d)
    if full:
        return {'heatmaps': hm, 'joints': torch.stack(joints), 'loss': float(loss), 'X': X}
    return X


def host_cores():
    """(cores this process may run on, the host's CPU count): the scheduler affinity, capped by a
    cgroup CPU quota when one is set (a GPU box gives each GPU's job a share of a larger host)."""
    host = os.cpu_count() or 1
    try:
        usable = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        usable = host
    try:
        with open('/sys/fs/cgroup/cpu.max') as f:
            quota, period = f.read().split()[:2]
        if quota != 'max':
            usable = min(usable, max(1, -(-int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return usable, host


def cpu_baseline(layers, size, groups, seconds):
    """The oracle chain on the host cores: the full configs[2] batch (groups x 4 frames,
    repeated until `seconds` have passed, at least once) and configs[0] (batch 1,
    forward only), on every core this process may use (host_cores).  Returns (cpu_baseline dict,
    the first full batch's oracle outputs)."""
    from models.pose_resnet import get_pose_net
    from oracle import pose_resnet_ref as PR
    from posu import synthetic as syn
    from posu.pipeline import synthetic_meta
    threads, host_cpus = host_cores()
    torch.set_num_threads(threads)
    net = get_pose_net(syn.make_cfg(num_layers=layers, image_size=size), is_train=False)
    sd = syn.synthetic_state_dict(net.state_dict(), seed=syn.calibrated_seed(layers, size),
                                  bn_stats=syn.load_bn_stats(layers, size))
    _, host = synthetic_meta(groups, 'cpu', image_size=size)
    views = syn.group_views(4, range(groups), size, seed=100)   # the bench's input batch 0
    frames, ref, t0 = 0, None, time.perf_counter()
    while True:
        out = oracle_chain(sd, layers, size, views, host, full=ref is None)
        ref = out if ref is None else ref
        frames += 4 * groups
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    x1 = syn.synthetic_views(1, 1, size, seed=7)[0]
    PR.pose_resnet_forward(x1, sd, layers)
    n1, t1 = 0, time.perf_counter()
    while n1 < 3 or time.perf_counter() - t1 < min(3.0, seconds / 4):
        PR.pose_resnet_forward(x1, sd, layers)
        n1 += 1
    c1_ms = (time.perf_counter() - t1) / n1 * 1e3
    ref['host'] = host
    return ({'value': round(frames / el, 3), 'unit': 'frames/s', 'cores': threads, 'host_cpus': host_cpus,
             'kind': 'port',
             'sample': '%d frames = %d pass(es) of the full %dx4 batch (R%d@%d) through the CPU oracle chain: '
                       'torch-CPU fp32 forward + soft-argmax + transform_back + FundamentalLoss + numpy DLT/SVD '
                       'triangulation, %.1f s' % (frames, frames // (4 * groups), groups, layers, size, el),
             'batch1_forward_ms': round(c1_ms, 2), 'batch1_frames_per_s': round(1e3 / c1_ms, 3)}, ref)


def compare_with_reference(out, ref, meta, dev):
    """The bench chain's outputs on its first input batch (heatmaps, image-px joints
    [V, G, J, 2], epipolar loss, X) against the CPU oracle chain's (the checker).

    * heatmaps / joints / loss: direct differences.
    * triangulation_same_2d: X from the device kernel vs the oracle's triangulation of the
      SAME device joints -- the triangulation's own parity (BASELINE's 1e-2 mm gate).
    * mpjpe (the bench line's mpjpe_vs_ref_mm): the pipeline's 2-D deviation from the
      reference chain, d = joints - joints_ref, laid on consistent geometry -- the
      synthetic 3-D poses projected into the group's cameras (p) -- and triangulated:
      device kernel on p + d against the oracle on p, per-joint error (mm) with
      run/test/test_triangulate.py:98-102's arithmetic.  The raw end-to-end X of a
      random-weight network is no measure: its four views' soft-argmax joints are
      mutually inconsistent, so the DLT solution sits near the plane at infinity and
      moves by metres for sub-pixel input changes (kept as raw_end_to_end for the record)."""
    from oracle import geometry_ref as G
    from posu import ops
    from posu.metrics import mpjpe_stats
    host = ref['host']
    V, ng, J = 4, ref['joints'].shape[1], ref['joints'].shape[2]
    hm_err = (out['hm0'] - ref['heatmaps']).abs()
    jerr = np.linalg.norm(out['coords0'] - ref['joints'].numpy(), axis=-1)
    p2d = out['coords0'].transpose(1, 0, 2, 3).reshape(ng * V, J, 2).astype(np.float64)
    tri = mpjpe_stats(out['X0'], G.triangulate_poses(host['cams'], p2d))
    proj = np.stack([np.stack([G.project_pose(host['poses3d'][g], host['cams'][g * V + v]) for g in range(ng)])
                     for v in range(V)])                                             # [V, G, J, 2]
    d = out['coords0'].astype(np.float64) - ref['joints'].numpy().astype(np.float64)
    Xb = ops.triangulate_dlt(meta.M, meta.intr, torch.from_numpy(proj + d).to(dev), None, undistort=True,
                             view_major=True).cpu().numpy()
    Xr = G.triangulate_poses(host['cams'], proj.transpose(1, 0, 2, 3).reshape(ng * V, J, 2))
    st = mpjpe_stats(Xb, Xr)
    raw = mpjpe_stats(out['X0'], ref['X'])
    r6 = lambda v: float('%.6g' % v)  # noqa: E731
    return {'mean': r6(st['mean']), 'std': r6(st['std']), 'max': r6(st['max']),
            'heatmap_abs_err': {'max': r6(hm_err.max()), 'mean': r6(hm_err.mean())},
            'joints_px_err': {'max': r6(jerr.max()), 'mean': r6(jerr.mean())},
            'epipolar_loss_rel_err': r6(abs(out['loss0'] / ref['loss'] - 1)),
            'triangulation_same_2d_mm': {'mean': r6(tri['mean']), 'max': r6(tri['max'])},
            'raw_end_to_end_mm': {'mean': r6(raw['mean']), 'max': r6(raw['max'])}}


# ------------------------------------------------------------------ inference
class Replayer:
    """Network and decode+geometry stages of one input batch, captured as two hipGraphs."""

    def __init__(self, plan, views, meta, groups, chunks, use_graph, dev):
        from posu import ops
        self.plan, self.views, self.meta, self.groups, self.chunks = plan, views, meta, groups, chunks
        self.ops = ops
        self.use_graph = use_graph
        self.dev = dev

    def stage_net(self):
        return self.plan.run(self.plan.pack_input(self.views), chunks=self.chunks, keep_features=False)[0]

    def stage_geo(self, hm):
        ops, meta = self.ops, self.meta
        coords = ops.softargmax2d(hm, beta=100.0, affine=meta.affines).view(4, self.groups, hm.shape[1], 2)
        loss = ops.epipolar_loss(coords, meta.weights, meta.F, meta.subj)
        X = ops.triangulate_dlt(meta.M, meta.intr, coords, None, undistort=True, view_major=True)
        return coords, loss, X

    def capture(self):
        s = torch.cuda.Stream(self.dev)
        s.wait_stream(torch.cuda.current_stream(self.dev))
        with torch.cuda.stream(s):
            for _ in range(2):
                self.stage_geo(self.stage_net())
        torch.cuda.current_stream(self.dev).wait_stream(s)
        torch.cuda.synchronize()
        self.g_net, self.g_geo = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.g_net):
            self.hm = self.stage_net()
        with torch.cuda.graph(self.g_geo, pool=self.g_net.pool()):
            self.out = self.stage_geo(self.hm)
        torch.cuda.synchronize()

    def run_net(self):
        if self.use_graph:
            self.g_net.replay()
            return self.hm
        self.hm = self.stage_net()
        return self.hm

    def run_geo(self, hm):
        if self.use_graph:
            self.g_geo.replay()
            return self.out
        self.out = self.stage_geo(hm)
        return self.out


def load_tiles(path):
    from posu import plan as pl
    with open(path) as f:
        table = json.load(f)
    for entry in table['tiles']:
        pl._TUNE_CACHE[tuple(_tup(entry['key']))] = entry['tile']
    return len(table['tiles'])


def _tup(x):
    return tuple(_tup(v) for v in x) if isinstance(x, list) else x


def save_tiles(path):
    from posu import plan as pl
    with open(path, 'w') as f:
        json.dump({'tiles': [{'key': list(k), 'tile': t} for k, t in pl.tuned_tiles().items()]}, f)


def rank_meta(args, rank, world, dev):
    """(shard, device metadata, host metadata) of this rank's groups of the global batch
    (args.groups per rank, posu.dist.shard_groups: the reference's DistributedSampler order)."""
    from posu import dist as pdist
    from posu.pipeline import subset_meta, synthetic_meta
    shard = pdist.shard_groups(args.groups * world, rank, world)
    meta, host = synthetic_meta(args.groups * world, dev, image_size=args.size)
    if world > 1:
        meta, host = subset_meta(meta, host, shard)
    return shard, meta, host


def time_pipeline(args, precision, dev, rank, steps, warmup, nbatch, autotune, dist=None, world=1):
    """Build, (auto)tune, capture and time the pipeline in one precision; returns a dict."""
    net = build_model(args.layers, args.size, precision, dev)
    shard, meta, host = rank_meta(args, rank, world, dev)
    plan = net.plan(dev)
    reps = [Replayer(plan, input_views(shard, args.size, b, dev), meta, len(shard), args.chunks,
                     not args.no_graph, dev) for b in range(nbatch)]
    tuned = None
    with torch.no_grad():
        for r in reps:  # eager warmup (plan packing, allocator)
            r.stage_geo(r.stage_net())
        torch.cuda.synchronize()
        if autotune:
            if args.tune_file and os.path.exists(args.tune_file):
                tuned = 'loaded %d layer tiles from %s' % (load_tiles(args.tune_file), args.tune_file)
            else:
                plan.autotune(plan.pack_input(reps[0].views), chunks=args.chunks, keep_features=False, reps=8)
                torch.cuda.synchronize()
                tuned = 'autotuned in-run'
                if args.tune_file:
                    save_tiles(args.tune_file)
        use_graph = not args.no_graph
        if use_graph:
            try:
                for r in reps:
                    r.capture()
            except Exception as e:  # report, then time eagerly
                print('graph capture failed (%s); timing eager launches' % e, file=sys.stderr)
                use_graph = False
                for r in reps:
                    r.use_graph = False
        for i in range(warmup):
            r = reps[i % nbatch]
            r.run_geo(r.run_net())
        stream = torch.cuda.current_stream(dev)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True),
               torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
        # decode + geometry of batch i on a second stream, overlapping the network of batch i + 1
        # (a two-stage pipeline over the rotated batches): batch i's geometry waits for its own
        # network; a batch's next network replay waits for its previous geometry (its graphs
        # share one memory pool and the heatmap buffer).  --serial-geo: one stream, in order.
        geo_stream = None if args.serial_geo or nbatch < 2 else torch.cuda.Stream(dev)
        geo_done = [None] * nbatch
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            b = i % nbatch
            r = reps[b]
            if geo_done[b] is not None:
                stream.wait_event(geo_done[b])
            ev[i][0].record(stream)
            hm = r.run_net()
            ev[i][1].record(stream)
            if geo_stream is None:
                ev[i][3].record(stream)
                r.run_geo(hm)
                ev[i][2].record(stream)
                continue
            geo_stream.wait_event(ev[i][1])
            ev[i][3].record(geo_stream)   # geometry starts: its own network done, the previous geometry too
            with torch.cuda.stream(geo_stream):
                r.run_geo(hm)
            ev[i][2].record(geo_stream)
            geo_done[b] = ev[i][2]
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        net_ms = float(np.mean([a.elapsed_time(b) for a, b, _, _ in ev]))
        geo_ms = float(np.mean([d.elapsed_time(c) for _, _, c, d in ev]))
        # the first batch's outputs, for the MPJPE check
        r = reps[0]
        coords, loss, X = r.run_geo(r.run_net())
        torch.cuda.synchronize()
    return {'elapsed': elapsed, 'net_ms': net_ms, 'geo_ms': geo_ms, 'X0': X.detach().cpu().numpy().copy(),
            'coords0': coords.detach().cpu().numpy().copy(), 'hm0': r.hm.detach().cpu().clone(),
            'use_graph': use_graph, 'tuned': tuned, 'loss0': float(loss), 'meta': r.meta, 'host': host,
            'shard': shard, 'chunks': args.chunks if args.chunks is not None else plan.default_chunks()}


def triangulation_parity_all_ranks(res, dev):
    """Every rank: the device triangulation of its groups' device joints against the oracle's
    triangulation of the SAME joints (the BASELINE 1e-2 mm gate, run/test/test_triangulate.py:98-102
    arithmetic), reduced over ranks with posu.dist (error sums and counts, max)."""
    from oracle import geometry_ref as G
    from posu import dist as pdist
    X0, c0 = res['X0'], res['coords0']
    V, ng, J = c0.shape[0], c0.shape[1], c0.shape[2]
    p2d = c0.transpose(1, 0, 2, 3).reshape(ng * V, J, 2).astype(np.float64)
    err = np.linalg.norm(X0 - G.triangulate_poses(res['host']['cams'], p2d), axis=-1)
    tot, cnt = pdist.sum_over_ranks([err.sum(), err.size], device=dev)
    mx = pdist.max_over_ranks(err.max(), device=dev)
    return {'mean': float('%.6g' % (tot / cnt)), 'max': float('%.6g' % mx), 'joints': int(cnt)}


def _json_default(o):
    """numpy values that reach the JSON line (arrays as lists, scalars as Python numbers); logged
    to stderr so the producing leg can be fixed."""
    import numpy as np
    if isinstance(o, np.ndarray):
        print('bench: numpy array of shape %s in the JSON line' % (o.shape,), file=sys.stderr)
        return o.tolist()
    if isinstance(o, np.generic):
        return o.item()
    if isinstance(o, torch.Tensor):
        print('bench: tensor of shape %s in the JSON line' % (tuple(o.shape),), file=sys.stderr)
        return o.tolist()
    raise TypeError('%s is not JSON serializable' % type(o).__name__)


def peaked_parity(args, dev):
    """tools/peaked.py: fit R50@256 to peaked targets through the (fp32) training path, then the fp32,
    fp16x3 (also with its tiles autotuned on the task, as the parity_mode leg tunes them), bf16 and
    fp16 chains against the CPU oracle chain on those weights (the checker leg; N = 1)."""
    sys.path.insert(0, os.path.join(REPO, 'tools'))
    import peaked
    t0 = time.perf_counter()
    net, task = peaked.fit_peaked(dev, steps=args.peaked_steps)
    torch.cuda.synchronize()
    fit_s = time.perf_counter() - t0
    out = {}
    ref = None
    # fp32 (the parity mode) first, then both 2-byte modes (same MFMA rate), the benched one included
    for prec in dict.fromkeys(('fp32', args.precision, 'fp16x3', 'bf16', 'fp16')):
        out[prec], ref = peaked.parity(net, task, dev, prec, ref)
    out['fp16x3_autotuned'], _ = peaked.parity(net, task, dev, 'fp16x3', ref, autotune=True)
    out['fit'] = {'steps': args.peaked_steps, 'seconds': round(fit_s, 2), 'groups': task['groups'], 'precision': 'fp32',
                  'heatmap_peak_mean': out['fp32']['heatmap_peak_mean'],
                  'oracle_mpjpe_vs_gt_mm': out['fp32']['oracle_mpjpe_vs_gt_mm']}
    return out


def time_configs1(args, dev, rank, world, dist):
    """BASELINE configs[1]: the ResNet-50 heatmap forward alone on a synthetic 256x256 batch of 64
    frames in bf16 (tiles autotuned for that batch, one hipGraph, HIP events on the launch
    stream): frames/s and the fraction of the bf16 MFMA peak."""
    from posu import synthetic as syn
    if (args.layers, args.size) != (50, 256):
        return None
    net = build_model(50, 256, 'bf16', dev)
    plan = net.plan(dev)
    views = [v.to(dev) for v in syn.synthetic_views(1, 64, 256, seed=300 + rank)]
    with torch.no_grad():
        run = lambda: plan.run(plan.pack_input(views), keep_features=False)[0]  # noqa: E731
        run()
        if not args.no_autotune:
            plan.autotune(plan.pack_input(views), keep_features=False, reps=8)
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            run()
        torch.cuda.current_stream(dev).wait_stream(s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            run()
        for _ in range(3):
            g.replay()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a.record()
        for _ in range(args.c1_steps):
            g.replay()
        b.record()
        torch.cuda.synchronize()
    ms = a.elapsed_time(b) / args.c1_steps
    from posu import dist as pdist
    ms_max = pdist.max_over_ranks(ms, device=dev)
    tf = GFLOP_PER_FRAME[(50, 256)] * 64 / (ms * 1e-3) / 1e3
    return {'metric': 'ResNet-50 heatmap forward frames/s (BASELINE configs[1]: synthetic 256x256 batch 64, bf16)',
            'value': round(64 * world / (ms_max * 1e-3), 2), 'unit': 'frames/s', 'network_ms': round(ms, 4),
            'replays': args.c1_steps, 'n_gpus': world,
            'roofline': {'bound': 'mfma', 'achieved': round(tf, 2), 'peak': PEAK_BF16_TFLOPS, 'unit': 'TFLOP/s',
                         'frac': round(tf / PEAK_BF16_TFLOPS, 4)}}


def _flags_off(flags, fn):
    """fn() with the posu.plan switches `flags` off; the plan switches and the autotuner's tables
    (the control plan re-tunes geometries it shares with the measured plan) restored afterwards."""
    from posu import plan as pl
    saved = {f: getattr(pl, f) for f in flags}
    tables = [(t, dict(t)) for t in (pl._TUNE_CACHE, pl._TUNE_TIMES, pl._REFINE_TIMES)]
    try:
        for f in flags:
            setattr(pl, f, False)
        return fn()
    finally:
        for f, v in saved.items():
            setattr(pl, f, v)
        for t, snap in tables:
            t.clear()
            t.update(snap)


def time_control(args, dev, rank, world, dist, precision=None, flags=CONTROL_FLAGS):
    """The benched pipeline (precision: the headline's, or another leg's) with `flags` off (the earlier
    round's plan), same process and box: its network_ms beside the leg's."""
    prec = precision or args.precision
    r = _flags_off(flags, lambda: time_pipeline(args, prec, dev, rank, args.control_steps, 3, args.batches,
                                                not args.no_autotune, dist, world))
    return {'flags_off': list(flags), 'precision': prec, 'network_ms': round(r['net_ms'], 4),
            'steps': args.control_steps, 'ms_per_step': round(r['elapsed'] / args.control_steps * 1e3, 4)}


def time_configs4(args, dev, rank, world, dist, steps=None):
    """BASELINE configs[4]'s per-GPU pipeline: R152 backbone at 384x384, fp16 compute, fp64
    triangulation, 16 groups x 4 views per GPU (the 8-GPU job's shard), tiles autotuned, the same
    two-stage replay as the line: frames/s and the fraction of the fp16 (= bf16) MFMA peak."""
    import argparse as _ap
    a4 = _ap.Namespace(**vars(args))
    a4.layers, a4.size, a4.groups, a4.precision, a4.tune_file = 152, 384, 16, 'fp16', ''
    steps = steps or args.c4_steps
    r = time_pipeline(a4, 'fp16', dev, rank, steps, 3, 2, not args.no_autotune, dist, world)
    from posu import dist as pdist
    el = pdist.max_over_ranks(r['elapsed'], device=dev)
    frames = 4 * a4.groups
    tf = GFLOP_PER_FRAME[(152, 384)] * frames / (r['net_ms'] * 1e-3) / 1e3
    return {'metric': '4-view 384x384 frames/sec (fwd+triangulate), R152 fp16 (BASELINE configs[4], per-GPU shard '
                      'of 16 groups x 4 views)', 'value': round(pdist.throughput(frames, steps, world, el), 2),
            'unit': 'frames/s', 'n_gpus': world, 'steps': steps, 'network_ms': round(r['net_ms'], 4),
            'ms_per_step': round(el / steps * 1e3, 4), 'dtype': 'fp16',
            'roofline': {'bound': 'mfma', 'achieved': round(tf, 2), 'peak': PEAK_BF16_TFLOPS, 'unit': 'TFLOP/s',
                         'frac': round(tf / PEAK_BF16_TFLOPS, 4),
                         'flop_per_launch': '%.2f GFLOP/frame x %d frames' % (GFLOP_PER_FRAME[(152, 384)], frames)}}


def infer_main(args):
    from posu import dist as pdist
    _, local, world = pdist.env_rank()
    dev, backend = rank_device(local)
    torch.cuda.set_device(dev)
    rank, local, world, dist = init_ranks(args, backend, device=dev)
    frames = 4 * args.groups
    res = time_pipeline(args, args.precision, dev, rank, args.steps, args.warmup, args.batches,
                        not args.no_autotune, dist, world)
    tri_all = triangulation_parity_all_ranks(res, dev)
    elapsed = pdist.max_over_ranks(res['elapsed'], device=dev)
    value = pdist.throughput(frames, args.steps, world, elapsed)
    per_rank = gather_per_rank([frames * args.steps, res['elapsed']], dist, device=dev)
    gf = GFLOP_PER_FRAME.get((args.layers, args.size))
    peak = PEAK_F32_TFLOPS if args.precision == 'fp32' else PEAK_BF16_TFLOPS  # fp16 (x3) dense peak == bf16
    roof = None
    if gf is not None:
        achieved = gf * frames / (res['net_ms'] * 1e-3) / 1e3  # TFLOP/s
        traffic, src = pmc_traffic(args.layers, args.size, args.precision, args.groups)
        roof = {'bound': 'mfma', 'achieved': round(achieved, 2), 'peak': peak, 'unit': 'TFLOP/s',
                'frac': round(achieved / peak, 4), 'traffic': traffic,
                'kernel': 'network per replay: fused stem (stem_pool_kernel) + fused layer1 Bottlenecks '
                          '(bottleneck64_kernel) + conv stack (conv_igemm / conv_persist kernels, fused deconv+head)',
                'flop_per_launch': '%.2f GFLOP/frame x %d frames' % (gf, frames)}
        if traffic:
            roof['traffic_source'] = dict(src, counters='PMC FETCH_SIZE x2 + WRITE_SIZE, bytes per forward')
            roof['hbm_floor_ms'] = round(traffic / 6.3e12 * 1e3, 4)  # at the ~6.3 TB/s achievable
        if (args.layers, args.size) == (50, 256) and args.precision in ('bf16', 'fp16'):
            # compulsory bytes of the same launches (posu.roofline: inputs, weights read once, outputs
            # written once); traffic / algorithmic = the forward's over-fetch
            from posu import roofline as _rl
            alg = _rl.r50_256_algorithmic_bytes(frames, 2)
            roof['algorithmic_bytes'] = alg
            if traffic:
                roof['traffic_over_algorithmic'] = round(traffic / alg, 4)
    # the training leg right after the headline leg, before the other legs (see DESIGN.md section 6:
    # behind the fp32 / configs1 legs the same step read 23.98 instead of 21.6 ms)
    def train_leg():
        if args.empty_cache_before_train:
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
        t = run_training(args, dev, rank, world, dist, args.train_steps, 3)
        tr = {k: t[k] for k in ('value', 'unit', 'ms_per_step', 'loss', 'steps', 'warmup')}
        roof = t['roofline'] or {}
        tr.update(metric=TRAIN_METRIC, n_gpus=world, frac=roof.get('frac'), traffic=roof.get('traffic'),
                  algorithmic_bytes=roof.get('algorithmic_bytes'),
                  traffic_over_algorithmic=roof.get('traffic_over_algorithmic'),
                  algorithmic_bytes_fused_bn=roof.get('algorithmic_bytes_fused_bn'),
                  traffic_over_fused_bn_ideal=roof.get('traffic_over_fused_bn_ideal'),
                  parallelism=t['config']['parallelism'], workload=t['config']['workload'],
                  optimizer=t['config']['optimizer'])
        return tr

    train = None
    if args.train_steps > 0 and not args.train_last:
        train = train_leg()
    fp32 = None
    if args.fp32_steps > 0 and args.precision != 'fp32':
        r32 = time_pipeline(args, 'fp32', dev, rank, args.fp32_steps, 2, args.batches, False, dist, world)
        el32 = pdist.max_over_ranks(r32['elapsed'], device=dev)
        fp32 = {'value': round(pdist.throughput(frames, args.fp32_steps, world, el32), 2), 'unit': 'frames/s',
                'network_ms': round(r32['net_ms'], 3), 'steps': args.fp32_steps,
                'roofline_frac_f32': (round(gf * frames / (r32['net_ms'] * 1e-3) / 1e3 / PEAK_F32_TFLOPS, 4)
                                      if gf else None)}
    par = None
    if args.parity_steps > 0 and args.precision != 'fp16x3':
        rp = time_pipeline(args, 'fp16x3', dev, rank, args.parity_steps, 3, args.batches, not args.no_autotune, dist,
                           world)
        elp = pdist.max_over_ranks(rp['elapsed'], device=dev)
        par = {'precision': 'fp16x3', 'value': round(pdist.throughput(frames, args.parity_steps, world, elp), 2),
               'unit': 'frames/s', 'network_ms': round(rp['net_ms'], 4), 'steps': args.parity_steps,
               'ms_per_step': round(elp / args.parity_steps * 1e3, 4), 'chunks': rp['chunks']}
        if gf:
            tfp = gf * frames / (rp['net_ms'] * 1e-3) / 1e3
            # frac: the network's real flops against the dense fp16 peak; mfma_frac: the MFMA work
            # issued (three fp16 products per multiply-add) against it
            par['roofline'] = {'bound': 'mfma', 'achieved': round(tfp, 2), 'peak': PEAK_BF16_TFLOPS,
                               'unit': 'TFLOP/s', 'frac': round(tfp / PEAK_BF16_TFLOPS, 4),
                               'mfma_frac': round(3 * tfp / PEAK_BF16_TFLOPS, 4)}
            ptr, psrc = pmc_traffic(args.layers, args.size, 'fp16x3', args.groups)
            if ptr:
                par['roofline']['traffic'] = ptr
                par['roofline']['traffic_source'] = dict(psrc, counters='PMC FETCH_SIZE x2 + WRITE_SIZE, bytes per forward')
        if args.control_steps > 0:
            par['control'] = time_control(args, dev, rank, world, dist, 'fp16x3', CONTROL_FLAGS_PARITY)
    c1 = time_configs1(args, dev, rank, world, dist) if args.c1_steps > 0 else None
    control = None
    if args.control_steps > 0:
        control = (time_control(args, dev, rank, world, dist) if CONTROL_FLAGS else
                   {'flags_off': [], 'note': 'no switch of the headline plan added this round; parity_mode.control '
                                             'and configs4.control time the legs whose plans changed'})
    c4 = time_configs4(args, dev, rank, world, dist) if args.c4_steps > 0 else None
    if c4 is not None and args.control_steps > 0:
        cc = _flags_off(CONTROL_FLAGS_C4, lambda: time_configs4(args, dev, rank, world, dist,
                                                                 steps=min(args.c4_steps, args.control_steps)))
        c4['control'] = {'flags_off': list(CONTROL_FLAGS_C4), 'network_ms': cc['network_ms'], 'value': cc['value']}
    if args.train_steps > 0 and args.train_last:
        train = train_leg()
    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return
    cpu, mpjpe, random_w = None, None, None
    if world == 1 and not (args.no_cpu_baseline and args.no_mpjpe):
        cpu, ref = cpu_baseline(args.layers, args.size, args.groups,
                                0.0 if args.no_cpu_baseline else args.cpu_baseline_seconds)
        if args.no_cpu_baseline:
            cpu = None
        if not args.no_mpjpe:
            random_w = compare_with_reference(res, ref, res['meta'], dev)
            random_w['what'] = ('%s pipeline vs the fp32 CPU oracle chain on the first input batch of the '
                                'random-weight network (flat heatmaps); mean/std/max: its 2-D joint deviation laid on '
                                'the synthetic poses\' projections and triangulated -- see bench.compare_with_reference'
                                % args.precision)
            if fp32 is not None:
                fp32['random_weight_chain_vs_ref'] = compare_with_reference(r32, ref, r32['meta'], dev)
            if par is not None:
                par['random_weight_chain_vs_ref'] = compare_with_reference(rp, ref, rp['meta'], dev)
    peaked = None
    if world == 1 and not args.no_mpjpe and args.peaked_steps > 0 and (args.layers, args.size) == (50, 256):
        peaked = peaked_parity(args, dev)
        mpjpe = dict(peaked[args.precision]['mpjpe_vs_ref_mm'])
        mpjpe['what'] = ('%s chain (eval plan -> soft-argmax + crop affine -> fp64 DLT) vs the fp32 CPU oracle chain '
                         'on a fitted R50@256 whose heatmaps peak (mean %.2f) where 8 synthetic 4-view poses project '
                         '(tools/peaked.py); per-joint 3-D error in mm, test_triangulate.py:98-101 arithmetic; '
                         'details in peaked_parity' % (args.precision, peaked['fit']['heatmap_peak_mean']))
        if par is not None:
            par['peaked_parity'] = {k: peaked['fp16x3'][k] for k in ('heatmap_abs_err', 'mpjpe_vs_ref_mm')}
            par['peaked_parity_autotuned'] = {k: peaked['fp16x3_autotuned'][k]
                                              for k in ('heatmap_abs_err', 'mpjpe_vs_ref_mm')}
            # BASELINE.json's bars (heatmaps 1e-3; triangulated joints 1e-2 mm, mean and max), with the
            # heuristic tiles and with the tuned ones
            par['within_baseline_bars'] = all(
                r['heatmap_abs_err']['max'] < 1e-3 and r['mpjpe_vs_ref_mm']['max'] < 1e-2 and
                r['mpjpe_vs_ref_mm']['mean'] < 1e-2 for r in (peaked['fp16x3'], peaked['fp16x3_autotuned']))
    line = {
        'metric': METRIC, 'value': round(value, 2), 'unit': 'frames/s', 'n_gpus': world, 'steps': args.steps,
        'warmup': args.warmup, 'ms_per_step': round(elapsed / args.steps * 1e3, 4), 'higher_is_better': True,
        'scaling': 'weak', 'vs_baseline': None, 'dtype': args.precision, 'data': 'synthetic',
        'config': {'workload': '4-view H36M-like batch %dx4 at %dx%d: PoseResNet-%d forward + soft-argmax/affine '
                               '+ epipolar loss + fp64 DLT triangulation (BASELINE configs[2])'
                               % (args.groups, args.size, args.size, args.layers),
                   'frames_per_gpu_step': frames, 'global_batch_frames': frames * world,
                   'parallelism': 'dp%d (the global batch of %d groups sharded by posu.dist.shard_groups, '
                                  'no data-path collective)' % (world, args.groups * world),
                   'hipgraph': res['use_graph'], 'chunks': res['chunks'], 'tiles': res['tuned'] or 'heuristic',
                   'input_batches_rotated': args.batches,
                   'stages': ('network and decode+geometry in order on one stream' if args.serial_geo or args.batches < 2
                              else 'network on the main stream, decode+geometry of the same batch on a second '
                                   'stream overlapping the next batch\'s network')},
        'network_ms': round(res['net_ms'], 4), 'decode_geometry_ms': round(res['geo_ms'], 4),
        'groups_per_s': round(value / 4, 2), 'per_rank_frames': [int(p[0]) for p in per_rank],
        'per_rank_seconds': [round(p[1], 5) for p in per_rank],
        'mpjpe_vs_ref_mm': mpjpe, 'peaked_parity': peaked,
        'random_weight_chain_vs_ref': random_w if world == 1 and not args.no_mpjpe else None,
        'triangulation_same_2d_mm_all_ranks': tri_all, 'fp32_mode': fp32, 'parity_mode': par,
        'configs1': c1, 'configs4': c4, 'control': control, 'train_mode': train,
        'roofline': roof, 'cpu_baseline': cpu,
    }
    if os.environ.get('POSU_SHARED_GPU_REHEARSAL') == '1':
        line['shared_gpu_rehearsal'] = 'ranks share GPUs over gloo: a plumbing rehearsal, not a measurement'
    print(json.dumps(line, default=_json_default))
    if dist is not None:
        dist.destroy_process_group()


# ------------------------------------------------------------------ training
# the benched step's weight of the epipolar (FundamentalLoss) term: the reference config's default
# config.LOSS.FUNDAMENTAL_LOSS_WEIGHT (lib/core/config.py:102; function.py:308-309 multiplies by it)
TRAIN_FUND_WEIGHT = 1.0


def train_batch(args, dev, rank=0, world=1, dist=None, fund_weight=None):
    """The configs[3] training batch of this rank and its loss (tests/test_gpu_train_full.py checks
    exactly this step): the bench's calibrated R50 (train mode, per-view BN) wrapped in
    MultiViewPose (DDP when dist is given), the rank's 4-view shard of synthetic crops, Gaussian
    targets at seeded positions, loss() = sum over views of JointsMSELoss + TRAIN_FUND_WEIGHT (or
    fund_weight) x the epipolar loss of the soft-argmax joints weighted by the target weights, as the
    reference's USE_TARGET_WEIGHT_FUND (core/function.py:154-366, 296-310).  Returns a dict."""
    fw = TRAIN_FUND_WEIGHT if fund_weight is None else fund_weight
    from posu import synthetic as syn
    from core.loss import JointsMSELoss, FundamentalLoss
    from models.multiview_pose_resnet import get_multiview_pose_net
    from utils.transforms import integral_preds_image_th
    from posu import ops
    cfg = syn.make_cfg(num_layers=args.layers, image_size=args.size)
    net = build_model(args.layers, args.size, args.precision, dev).train()
    model = get_multiview_pose_net(net, cfg)
    if dist is not None:
        local = dev.index
        model = torch.nn.parallel.DistributedDataParallel(model, device_ids=[local], output_device=local,
                                                          bucket_cap_mb=64)
    nb, nv, hs = args.groups, 4, args.size // 4
    shard, meta, host = rank_meta(args, rank, world, dev)
    views = input_views(shard, args.size, 0, dev)
    g = torch.Generator().manual_seed(7 + rank)
    ys, xs = torch.meshgrid(torch.arange(hs, dtype=torch.float32), torch.arange(hs, dtype=torch.float32),
                            indexing='ij')
    c = torch.rand(nv * nb, 16, 2, generator=g) * (hs - 8) + 4
    target = torch.exp(-((ys - c[..., 1, None, None]) ** 2 + (xs - c[..., 0, None, None]) ** 2) / 8.0).to(dev)
    target = target.view(nv, nb, 16, hs, hs)
    weight = torch.ones(nb, 16, 1, device=dev)
    fweight = weight.view(1, nb, 16).expand(nv, nb, 16).contiguous()   # the views' target weights [V, N, J]
    mse = JointsMSELoss(use_target_weight=True)
    fund = FundamentalLoss(cfg, fundamental_matrix_dict=syn.fundamental_dict(), device=dev)
    out = {'net': net, 'model': model, 'views': views, 'target': target, 'weight': weight, 'meta': meta,
           'host': host, 'F': fund.F}

    def loss_fn():
        raw, _, _, _ = model(views)
        loss = 0
        for v in range(nv):
            loss = loss + mse(raw[v], target[v], weight)
        coords = integral_preds_image_th(torch.cat(raw, 0), meta.affines).view(nv, nb, 16, 2)
        epi = ops.epipolar_loss(coords, fweight, fund.F, meta.subj)
        out['last'] = (raw, loss, epi)
        return loss + fw * epi
    out['loss'] = loss_fn
    return out


def run_training(args, dev, rank, world, dist, steps, warmup):
    """configs[3]: one training step = 4-view batch (groups x 4 frames per GPU) through the
    reference's step (core/function.py:154-366): train-mode forward with per-view BN,
    JointsMSELoss per view + FundamentalLoss on soft-argmax coords, backward, Adam.
    world > 1: DistributedDataParallel over RCCL (gradient all-reduce overlapped with the staged
    backward), weak scaling.  Returns the training line (a dict)."""
    tb = train_batch(args, dev, rank, world, dist)
    net, nv, nb = tb['net'], 4, args.groups
    # the reference's optimizer (utils.py:79-83: optim.Adam, same hyper-parameters); fused=True
    # runs the update as one kernel per parameter group instead of torch's foreach multi-tensor
    # launches (same math): 26.3 -> 22.8 ms per step measured A/B
    if args.adam == 'posu':   # the same update on the HIP kernel (posu_adam_step), state layout unchanged
        from posu.optim import Adam as PosuAdam
        opt = PosuAdam(net.parameters(), lr=1e-3)
    else:
        opt = torch.optim.Adam(net.parameters(), lr=1e-3, fused=args.adam == 'fused')

    def step():
        loss = tb['loss']()
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        return loss

    from posu import plan as pplan
    # POSU_STREAM_SKIP=k (diagnostic): take k streams from torch's pool first, as earlier legs of a
    # process do -- the training plan's weight-gradient side stream is the next pool stream
    for _ in range(int(os.environ.get('POSU_STREAM_SKIP', '0'))):
        torch.cuda.Stream(dev)
    stream = torch.cuda.Stream(dev, priority=-1) if args.train_stream == 'high' else torch.cuda.current_stream(dev)
    stream.wait_stream(torch.cuda.current_stream(dev))   # inputs / parameters made on the default stream
    with torch.cuda.stream(stream):
        return _train_loop(args, dev, dist, world, step, steps, warmup, nv, nb, stream)


def _train_loop(args, dev, dist, world, step, steps, warmup, nv, nb, stream):
    from posu import dist as pdist
    from posu import plan as pplan
    if not args.no_autotune:  # the first warm-up step times every admissible tile per conv geometry
        pplan._Tuner.active, pplan._Tuner.reps = True, 3
        try:
            step()
        finally:
            pplan._Tuner.active = False
    for _ in range(max(1, warmup)):
        step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    per_rank = gather_per_rank([nv * nb * steps, elapsed], dist, device=dev)
    elapsed = pdist.max_over_ranks(elapsed, device=dev)
    frames = nv * nb
    value = pdist.throughput(frames, steps, world, elapsed)
    gf = TRAIN_GFLOP_PER_FRAME.get((args.layers, args.size))
    roof = None
    if gf is not None:
        achieved = gf * value / world / 1e3
        peak = PEAK_F32_TFLOPS if args.precision == 'fp32' else PEAK_BF16_TFLOPS
        traffic, src = pmc_traffic_train(args.layers, args.size, args.precision, nb)
        roof = {'bound': 'mfma', 'achieved': round(achieved, 2), 'peak': peak, 'unit': 'TFLOP/s',
                'frac': round(achieved / peak, 4), 'traffic': traffic,
                'kernel': 'whole training step per GPU (fwd + bwd convs, BN, Adam)',
                'flop_per_launch': '%.1f GFLOP/frame x %d frames' % (gf, frames)}
        if traffic:
            roof['traffic_source'] = dict(src, counters='PMC FETCH_SIZE x2 + WRITE_SIZE, bytes per training step')
            roof['hbm_floor_ms'] = round(traffic / 6.3e12 * 1e3, 4)  # at the ~6.3 TB/s achievable
        if (args.layers, args.size, args.precision) == (50, 256, 'bf16'):
            # every tensor once per launch of the step's classes (posu/roofline.py); traffic /
            # algorithmic = the step's over-fetch (batchnorm's four passes are in the floor: it
            # prices the launch structure, the fusions are DESIGN.md's)
            from posu import roofline as _rl
            alg = _rl.r50_256_train_algorithmic_bytes(frames, 2)
            roof['algorithmic_bytes'] = alg
            # beside it the ideal step with BatchNorm fused into its neighbours (round 6): what the
            # separate BN passes cost, in bytes
            ideal = _rl.r50_256_train_algorithmic_bytes(frames, 2, fused_bn=True)
            roof['algorithmic_bytes_fused_bn'] = ideal
            if traffic and nb == 32:
                roof['traffic_over_algorithmic'] = round(traffic / alg, 4)
                roof['traffic_over_fused_bn_ideal'] = round(traffic / ideal, 4)
    return {
        'metric': TRAIN_METRIC, 'value': round(value, 2), 'unit': 'frames/s', 'n_gpus': world,
        'steps': steps, 'warmup': warmup, 'ms_per_step': round(elapsed / steps * 1e3, 4),
        'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None, 'dtype': args.precision,
        'data': 'synthetic',
        'config': {'workload': '4-view batch %dx4 at %dx%d: PoseResNet-%d train step (per-view BN, '
                               'JointsMSE + FundamentalLoss, Adam) (BASELINE configs[3])'
                               % (nb, args.size, args.size, args.layers),
                   'frames_per_gpu_step': frames, 'global_batch_frames': frames * world,
                   'parallelism': 'dp%d (DistributedDataParallel, RCCL gradient all-reduce overlapped with the '
                                  'staged backward)' % world,
                   'optimizer': 'Adam lr 1e-3 (%s)' % args.adam},
        'per_rank_frames': [int(p[0]) for p in per_rank],
        'loss': round(float(loss.detach()), 5), 'roofline': roof, 'cpu_baseline': None,
    }


def train_main(args):
    """`--mode train`: the configs[3] training step as the bench line."""
    from posu import dist as pdist
    _, local, _ = pdist.env_rank()
    dev, backend = rank_device(local)
    torch.cuda.set_device(dev)
    rank, local, world, dist = init_ranks(args, backend, device=dev)
    line = run_training(args, dev, rank, world, dist, args.steps, args.warmup)
    if rank == 0:
        print(json.dumps(line, default=_json_default))
    if dist is not None:
        dist.destroy_process_group()


def dump_tiles():
    """POSU_DUMP_TILES=path: the process's autotuned tile table (every leg) as JSON, for diffing
    the tile choices of two runs."""
    path = os.environ.get('POSU_DUMP_TILES')
    if path:
        from posu import plan as pl
        times, ctx = pl.tuning_times(), pl.refine_times()
        with open(path, 'w') as f:
            json.dump(sorted([[repr(k), t, {str(c): round(ms, 4) for c, ms in times.get(k, {}).items()},
                               {str(c): round(ms, 4) for c, ms in ctx.get(k, {}).items()}]
                              for k, t in pl.tuned_tiles().items()]), f, indent=0)


def main():
    args = parse()
    if args.gpus > 1 and 'WORLD_SIZE' not in os.environ:
        sys.exit(spawn_ranks(args))   # before anything touches the GPU
    if args.dry_run:
        return dry_run_main(args)
    apply_plan_flags(args.plan_flag)
    try:
        if args.mode == 'train':
            return train_main(args)
        return infer_main(args)
    finally:
        dump_tiles()


if __name__ == '__main__':
    main()
