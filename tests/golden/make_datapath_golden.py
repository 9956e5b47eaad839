"""Golden for the data-path kernels: the REFERENCE's
JointsDatasetCompatible.generate_heatmap (lib/dataset/joints_dataset_compatible.py,
imported in-process with stand-ins for cv2 / torchvision, which are not installed and
which generate_heatmap does not use) called per sample on seeded joints, and the
integral decode of run/test/test_integral.py:63-70 (a script: its lines are restated
here as numpy on seeded heatmaps).  Run once in this container:

    python tests/golden/make_datapath_golden.py
"""
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def datapath_inputs(seed=0):
    r = np.random.default_rng(seed)
    n, j = 6, 16
    joints = r.uniform(-20, 276, size=(n, j, 2)).astype(np.float32)
    joints[0, :4] = [[0.0, 0.0], [255.9, 255.9], [-13.0, 100.0], [270.0, 5.0]]   # corners / just outside
    joints[1, :3] = [[-2.1, -1.7], [1.9, 2.2], [258.0, 258.0]]                    # int() truncation at < 0
    vis = (r.uniform(size=(n, j)) > 0.2).astype(np.float32)
    sources = np.array(['mpii', 'h36m', 'mpii', 'h36m', 'mpii', 'mpii'])
    hm = np.abs(r.standard_normal((4, j, 64, 64))).astype(np.float32)
    return joints, vis, sources, hm


def main():
    sys.path.insert(0, '/root/reference/lib')
    sys.modules.setdefault('cv2', types.ModuleType('cv2'))
    tv = types.ModuleType('torchvision')
    tv.transforms = types.ModuleType('torchvision.transforms')
    sys.modules.setdefault('torchvision', tv)
    sys.modules.setdefault('torchvision.transforms', tv.transforms)
    # the module file itself (the dataset package __init__ pulls in json_tricks etc.)
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        'ref_joints_dataset_compatible', '/root/reference/lib/dataset/joints_dataset_compatible.py')
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    JointsDatasetCompatible = mod.JointsDatasetCompatible
    joints, vis, sources, hm = datapath_inputs()
    stub = types.SimpleNamespace(num_joints=16, heatmap_size=np.array([64, 64]), image_size=np.array([256, 256]),
                                 sigma=2, pseudo_label=False)
    targets, weights = [], []
    for n in range(joints.shape[0]):
        jv = np.stack([vis[n], vis[n]], axis=1)
        t, w = JointsDatasetCompatible.generate_heatmap(stub, joints[n].copy(), jv, sources[n])
        targets.append(t)
        weights.append(w)
    # test_integral.py:63-70
    h = hm / np.sum(hm, axis=(2, 3), keepdims=True)
    coordinates = np.arange(64).reshape((1, 1, 64))
    accu_w = np.sum(h, axis=2)
    accu_h = np.sum(h, axis=3)
    integral = np.stack((np.sum(accu_w * coordinates, axis=2), np.sum(accu_h * coordinates, axis=2)), axis=2)
    np.savez_compressed(os.path.join(HERE, 'datapath.npz'), targets=np.stack(targets), weights=np.stack(weights),
                        integral=integral)
    print('datapath golden written', np.stack(weights).sum())


if __name__ == '__main__':
    main()
