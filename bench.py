"""Benchmark of the 4-view hot path (BASELINE.json metric: 4-view 256x256 frames/sec,
fwd + triangulate).

One step = one batch of 32 groups x 4 views (128 frames, 256x256, synthetic N(0,1)
crops already resident in HBM) through
    PoseResNet-50 forward (bf16 MFMA kernels) -> soft-argmax + crop affine
    -> epipolar loss -> fp64 DLT triangulation,
captured as two hipGraphs (network | decode+geometry) and replayed.  With --gpus N
(launched by torch.distributed.run) every rank processes its own 32 groups (weak
scaling, no data-path collective); time = max over ranks.

Also reported, on the same JSON line:
  roofline     -- the conv stack (implicit-GEMM MFMA kernels): 14.47 GFLOP/frame x 128
                  frames per network replay / its HIP-event time, against the dense bf16
                  MFMA peak (2.5 PFLOP/s);
  cpu_baseline -- the CPU oracle (torch-CPU fp32 restatement of the reference path + the
                  numpy pymvg-style triangulation) timed on the host cores on a bounded
                  sample, rank 0 at N = 1 only.
"""
import argparse
import json
import os
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
    ap.add_argument('--layers', type=int, default=50)
    ap.add_argument('--size', type=int, default=256)
    ap.add_argument('--precision', default='bf16', choices=['bf16', 'fp16', 'fp32'])
    ap.add_argument('--no-graph', action='store_true')
    ap.add_argument('--no-autotune', action='store_true', help='keep the built-in conv tile heuristic')
    ap.add_argument('--chunks', type=int, default=1,
                    help='depth-first slices for the HBM-bound stem..layer2 / deconv2..head stages')
    ap.add_argument('--cpu-baseline-seconds', type=float, default=12.0)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    return ap.parse_args()


def build_model(layers, size, precision, device):
    from models.pose_resnet import get_pose_net
    from posu import synthetic as syn
    net = get_pose_net(syn.make_cfg(num_layers=layers, image_size=size), is_train=False, precision=precision)
    net.load_state_dict(syn.synthetic_state_dict(net.state_dict(), seed=0, bn_stats=syn.load_bn_stats(layers, size)))
    return net.to(device).eval()


def pmc_traffic(layers, size, precision, groups):
    """HBM bytes of one network forward from the newest committed PMC reduction
    (profiles/<round>/pmc_traffic_network.txt, tools/profile_round.sh), for the default
    workload it was measured on; None otherwise."""
    if (layers, size, precision, groups) != (50, 256, 'bf16', 32):
        return None, None
    import glob
    files = sorted(glob.glob(os.path.join(REPO, 'profiles', 'r*', 'pmc_traffic_network.txt')))
    if not files:
        return None, None
    with open(files[-1]) as f:
        d = json.loads(f.readline())
    return d['traffic_bytes'], os.path.relpath(files[-1], REPO)


def cpu_baseline(layers, size, seconds):
    """Oracle chain on the host cores for a bounded sample of the same workload."""
    from oracle import geometry_ref as G
    from oracle import pose_resnet_ref as PR
    from models.pose_resnet import get_pose_net
    from posu import synthetic as syn
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    net = get_pose_net(syn.make_cfg(num_layers=layers, image_size=size), is_train=False)
    sd = syn.synthetic_state_dict(net.state_dict(), seed=0, bn_stats=syn.load_bn_stats(layers, size))
    ng = 1  # one 4-view group per iteration
    meta_host = _cpu_meta(ng, size)
    views = syn.synthetic_views(4, ng, size, seed=0)
    x = torch.cat(views, 0)

    def one():
        hm, _, _ = PR.pose_resnet_forward(x, sd, layers)
        sa = G.softargmax2d(hm)
        img = G.transform_back(sa, meta_host['centers'], meta_host['scales'], [size // 4, size // 4])
        joints = [img[v * ng:(v + 1) * ng] for v in range(4)]
        G.fundamental_loss(joints, [torch.ones(ng, 16, 1)] * 4, meta_host['subjects'], meta_host['F_dict'])
        p2d = torch.stack(joints, 1).reshape(ng * 4, 16, 2).double().numpy()
        G.triangulate_poses(meta_host['cams'], p2d)
    one()
    frames, t0 = 0, time.perf_counter()
    while True:
        one()
        frames += 4 * ng
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {'value': frames / el, 'unit': 'frames/s', 'cores': threads, 'kind': 'port',
            'sample': '%d frames (%d 4-view groups, 1 group per iteration) of the same R%d@%d workload through '
                      'the CPU oracle: torch-CPU fp32 forward + soft-argmax + transform_back + FundamentalLoss + '
                      'numpy DLT/SVD triangulation, %.1f s' % (frames, frames // 4, layers, size, el)}


def _cpu_meta(ng, size):
    from posu import synthetic as syn
    from multiviews.cameras import project_pose
    cams = syn.group_cameras(ng)
    poses = syn.synthetic_poses3d(ng)
    centers = np.zeros((4 * ng, 2))
    for g in range(ng):
        for v in range(4):
            centers[v * ng + g] = project_pose(poses[g, :1], cams[g * 4 + v])[0]
    return {'cams': cams, 'centers': centers, 'scales': np.full((4 * ng, 2), 5.0),
            'subjects': syn.group_subjects(ng), 'F_dict': syn.fundamental_dict()}


def train_main(args):
    """configs[3]: one training step = 4-view batch (groups x 4 frames per GPU) through the
    reference's step (core/function.py:154-366): train-mode forward with per-view BN,
    JointsMSELoss per view + FundamentalLoss on soft-argmax coords, backward, Adam.
    N > 1: DistributedDataParallel over RCCL (gradient all-reduce), weak scaling."""
    from posu import dist as pdist
    from posu import synthetic as syn
    from posu.pipeline import synthetic_meta
    from core.loss import JointsMSELoss, FundamentalLoss
    from models.multiview_pose_resnet import get_multiview_pose_net
    from utils.transforms import integral_preds_image_th
    rank, local, world = pdist.env_rank()
    dev = torch.device('cuda', local)
    torch.cuda.set_device(dev)
    dist = None
    if world > 1:
        import torch.distributed as dist
        pdist.init('nccl', device=dev)
    cfg = syn.make_cfg(num_layers=args.layers, image_size=args.size)
    net = build_model(args.layers, args.size, args.precision, dev).train()
    model = get_multiview_pose_net(net, cfg)
    if dist is not None:
        model = torch.nn.parallel.DistributedDataParallel(model, device_ids=[local], output_device=local,
                                                          bucket_cap_mb=64)
    nb, nv, hs = args.groups, 4, args.size // 4
    views = [v.to(dev) for v in syn.synthetic_views(nv, nb, args.size, seed=100 + rank)]
    meta, _ = synthetic_meta(nb, dev, image_size=args.size)
    g = torch.Generator().manual_seed(7 + rank)
    ys, xs = torch.meshgrid(torch.arange(hs, dtype=torch.float32), torch.arange(hs, dtype=torch.float32),
                            indexing='ij')
    c = torch.rand(nv * nb, 16, 2, generator=g) * (hs - 8) + 4
    target = torch.exp(-((ys - c[..., 1, None, None]) ** 2 + (xs - c[..., 0, None, None]) ** 2) / 8.0).to(dev)
    target = target.view(nv, nb, 16, hs, hs)
    weight = torch.ones(nb, 16, 1, device=dev)
    mse = JointsMSELoss(use_target_weight=True)
    fund = FundamentalLoss(cfg, fundamental_matrix_dict=syn.fundamental_dict(), device=dev)
    opt = torch.optim.Adam(net.parameters(), lr=1e-3)
    subj = meta.subj

    def step():
        raw, _, _, _ = model(views)
        loss = 0
        for v in range(nv):
            loss = loss + mse(raw[v], target[v], weight)
        coords = integral_preds_image_th(torch.cat(raw, 0), meta.affines).view(nv, nb, 16, 2)
        from posu import ops
        loss = loss + 1e-3 * ops.epipolar_loss(coords, None, fund.F, subj)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        return loss

    for _ in range(max(1, args.warmup)):
        step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    elapsed = pdist.max_over_ranks(elapsed, device=dev)
    frames = nv * nb
    value = pdist.throughput(frames, args.steps, world, elapsed)
    gf = TRAIN_GFLOP_PER_FRAME.get((args.layers, args.size))
    roof = None
    if gf is not None:
        achieved = gf * value / world / 1e3
        peak = PEAK_F32_TFLOPS if args.precision == 'fp32' else PEAK_BF16_TFLOPS
        roof = {'bound': 'mfma', 'achieved': round(achieved, 2), 'peak': peak, 'unit': 'TFLOP/s',
                'frac': round(achieved / peak, 4), 'traffic': None,
                'kernel': 'whole training step per GPU (fwd + bwd convs, BN, Adam)',
                'flop_per_launch': '%.1f GFLOP/frame x %d frames' % (gf, frames)}
    if rank == 0:
        line = {
            'metric': TRAIN_METRIC, 'value': round(value, 2), 'unit': 'frames/s', 'n_gpus': world,
            'steps': args.steps, 'warmup': args.warmup, 'ms_per_step': round(elapsed / args.steps * 1e3, 4),
            'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None, 'dtype': args.precision,
            'data': 'synthetic',
            'config': {'workload': '4-view batch %dx4 at %dx%d: PoseResNet-%d train step (per-view BN, '
                                   'JointsMSE + FundamentalLoss, Adam) (BASELINE configs[3])'
                                   % (nb, args.size, args.size, args.layers),
                       'frames_per_gpu_step': frames, 'global_batch_frames': frames * world,
                       'parallelism': 'dp%d (DistributedDataParallel, RCCL gradient all-reduce)' % world},
            'loss': round(float(loss), 5), 'roofline': roof, 'cpu_baseline': None,
        }
        print(json.dumps(line))
    if dist is not None:
        dist.destroy_process_group()


def main():
    args = parse()
    if args.mode == 'train':
        return train_main(args)
    from posu import dist as pdist
    rank, local, world = pdist.env_rank()
    dev = torch.device('cuda', local)
    torch.cuda.set_device(dev)
    dist = None
    if world > 1:
        import torch.distributed as dist
        pdist.init('nccl', device=dev)

    from posu import synthetic as syn
    from posu.pipeline import synthetic_meta
    from posu import ops

    net = build_model(args.layers, args.size, args.precision, dev)
    meta, _ = synthetic_meta(args.groups, dev, image_size=args.size)
    views = [v.to(dev) for v in syn.synthetic_views(4, args.groups, args.size, seed=100 + rank)]
    plan = net.plan(dev)
    frames = 4 * args.groups

    # two stages so the network can be timed on its own with events between replays
    def stage_net():
        return plan.run(plan.pack_input(views), chunks=args.chunks, keep_features=False)[0]

    def stage_geo(hm):
        coords = ops.softargmax2d(hm, beta=100.0, affine=meta.affines).view(4, args.groups, hm.shape[1], 2)
        loss = ops.epipolar_loss(coords, meta.weights, meta.F, meta.subj)
        X = ops.triangulate_dlt(meta.M, meta.intr, coords, None, undistort=True, view_major=True)
        return coords, loss, X

    with torch.no_grad():
        for _ in range(3):  # eager warmup (plan packing, allocator)
            hm = stage_net()
            stage_geo(hm)
        torch.cuda.synchronize()
        if not args.no_autotune:  # per-layer conv tile choice, timed on the real operands
            plan.autotune(plan.pack_input(views), chunks=args.chunks, keep_features=False, reps=8)
            torch.cuda.synchronize()
        use_graph = not args.no_graph
        if use_graph:
            try:
                s = torch.cuda.Stream(dev)
                s.wait_stream(torch.cuda.current_stream(dev))
                with torch.cuda.stream(s):
                    for _ in range(2):
                        hm = stage_net()
                        stage_geo(hm)
                torch.cuda.current_stream(dev).wait_stream(s)
                torch.cuda.synchronize()
                g_net, g_geo = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
                with torch.cuda.graph(g_net):
                    hm_static = stage_net()
                with torch.cuda.graph(g_geo, pool=g_net.pool()):
                    out_static = stage_geo(hm_static)
                torch.cuda.synchronize()
            except Exception as e:  # report, then time eagerly
                print('graph capture failed (%s); timing eager launches' % e, file=sys.stderr)
                use_graph = False

        def run_net():
            if use_graph:
                g_net.replay()
                return hm_static
            return stage_net()

        def run_geo(hm):
            if use_graph:
                g_geo.replay()
                return out_static
            return stage_geo(hm)

        for _ in range(args.warmup):
            run_geo(run_net())
        stream = torch.cuda.current_stream(dev)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True),
               torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(args.steps):
            ev[i][0].record(stream)
            hm = run_net()
            ev[i][1].record(stream)
            run_geo(hm)
            ev[i][2].record(stream)
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        net_ms = float(np.mean([a.elapsed_time(b) for a, b, _ in ev]))
        geo_ms = float(np.mean([b.elapsed_time(c) for _, b, c in ev]))

    elapsed = pdist.max_over_ranks(elapsed, device=dev)
    value = pdist.throughput(frames, args.steps, world, elapsed)
    gf = GFLOP_PER_FRAME.get((args.layers, args.size))
    peak = PEAK_F32_TFLOPS if args.precision == 'fp32' else PEAK_BF16_TFLOPS  # fp16 dense peak == bf16
    roof = None
    if gf is not None:
        achieved = gf * frames / (net_ms * 1e-3) / 1e3  # TFLOP/s
        traffic, src = pmc_traffic(args.layers, args.size, args.precision, args.groups)
        roof = {'bound': 'mfma', 'achieved': round(achieved, 2), 'peak': peak, 'unit': 'TFLOP/s',
                'frac': round(achieved / peak, 4), 'traffic': traffic,
                'kernel': 'network per replay: fused stem (stem_pool_kernel) + conv stack (conv_igemm / conv_persist kernels, fused deconv+head)',
                'flop_per_launch': '%.2f GFLOP/frame x %d frames' % (gf, frames)}
        if traffic:
            roof['traffic_source'] = src + ' (PMC FETCH_SIZE x2 + WRITE_SIZE, bytes per forward)'
            roof['hbm_floor_ms'] = round(traffic / 6.3e12 * 1e3, 4)  # at the ~6.3 TB/s achievable
    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.layers, args.size, args.cpu_baseline_seconds)
    line = {
        'metric': METRIC, 'value': round(value, 2), 'unit': 'frames/s', 'n_gpus': world, 'steps': args.steps,
        'warmup': args.warmup, 'ms_per_step': round(elapsed / args.steps * 1e3, 4), 'higher_is_better': True,
        'scaling': 'weak', 'vs_baseline': None, 'dtype': args.precision, 'data': 'synthetic',
        'config': {'workload': '4-view H36M-like batch %dx4 at %dx%d: PoseResNet-%d forward + soft-argmax/affine '
                               '+ epipolar loss + fp64 DLT triangulation (BASELINE configs[2])'
                               % (args.groups, args.size, args.size, args.layers),
                   'frames_per_gpu_step': frames, 'global_batch_frames': frames * world,
                   'parallelism': 'dp%d (independent group shards, no data-path collective)' % world,
                   'hipgraph': use_graph, 'chunks': args.chunks, 'autotuned_tiles': not args.no_autotune},
        'network_ms': round(net_ms, 4), 'decode_geometry_ms': round(geo_ms, 4),
        'groups_per_s': round(value / 4, 2),
        'roofline': roof, 'cpu_baseline': cpu,
    }
    print(json.dumps(line))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
