"""The CPU baseline's restatement (oracle/pose_resnet_ref.py, bench.py's cpu_baseline leg)
against the reference's own PoseResNet module (imported from /root/reference/lib, CPU torch)
on the same weights and inputs: R50@256 eval forward at batch 1 (SURVEY §8(d)'s C1) and
batch 8, median of repeated runs, same thread count.  Runs in the build container only (the
reference does not exist on the GPU box); output: profiles/<round>/cpu_restatement_vs_reference.txt.

    python tools/cpu_ref_speed.py [--threads 8] [--reps 5]
"""
import argparse
import importlib.util
import os
import statistics
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--threads', type=int, default=8)
    ap.add_argument('--reps', type=int, default=5)
    a = ap.parse_args()
    torch.set_num_threads(a.threads)
    gold = _load('make_golden', os.path.join(REPO, 'tests', 'golden', 'make_golden.py'))
    ref_pr = gold._import_reference()[0]
    sys.path.insert(0, REPO)
    from oracle import pose_resnet_ref as PR
    syn = gold.syn
    cfg = syn.make_cfg(num_layers=50, image_size=256)
    block, layers = ref_pr.resnet_spec[50]
    net = ref_pr.PoseResNet(block, layers, cfg)
    sd = syn.synthetic_state_dict(net.state_dict(), seed=0, bn_stats=syn.load_bn_stats(50, 256))
    net.load_state_dict(sd)
    net.eval()
    print('threads %d, R50@256 eval forward, median of %d runs' % (a.threads, a.reps))
    for batch in (1, 8):
        x = torch.cat(syn.synthetic_views(1, batch, 256, seed=3), 0)
        ts = {'reference module': [], 'restatement (oracle)': []}
        with torch.no_grad():
            hr = net(x)[0]
            ho = PR.pose_resnet_forward(x, sd, 50)[0]
            for _ in range(a.reps):
                t0 = time.perf_counter()
                net(x)
                ts['reference module'].append(time.perf_counter() - t0)
                t0 = time.perf_counter()
                PR.pose_resnet_forward(x, sd, 50)
                ts['restatement (oracle)'].append(time.perf_counter() - t0)
        med = {k: statistics.median(v) for k, v in ts.items()}
        print('batch %d: reference %.1f ms, restatement %.1f ms, ratio %.3f; heatmaps max |diff| %.2e'
              % (batch, med['reference module'] * 1e3, med['restatement (oracle)'] * 1e3,
                 med['restatement (oracle)'] / med['reference module'], float((hr - ho).abs().max())))


if __name__ == '__main__':
    main()
