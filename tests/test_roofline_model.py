"""The algorithmic-bytes models bench.py divides PMC traffic by (posu/roofline.py) and the PMC
reduction of the training step (tools/pmc_train_traffic.py) on a synthetic counter CSV."""
import csv
import json
import os
import subprocess
import sys

import pytest

from posu import roofline as R

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_inference_launch_list():
    launches = R.r50_256_launches()
    assert len(launches) == 30
    assert R.r50_256_algorithmic_bytes() == sum(r + w for _, r, w in launches)
    # the f32 input dominates the stem; every launch reads and writes something
    assert all(r > 0 and w > 0 for _, r, w in launches)


def test_training_classes():
    c = R.r50_256_train_classes()
    total = R.r50_256_train_algorithmic_bytes()
    assert total == sum(r + w for r, w in c.values())
    # batchnorm's four passes over every conv output are the largest class
    assert max(c, key=lambda k: sum(c[k])) == 'batchnorm'
    # activations dominate: doubling the frames nearly doubles the bytes (weights / Adam fixed)
    assert 1.95 < R.r50_256_train_algorithmic_bytes(256) / total < 2.0
    # Adam: 7 f32 words per parameter (PoseResNet-50: ~34M parameters)
    nparam = sum(c['adam']) / 28
    assert 3.3e7 < nparam < 3.5e7


def test_pmc_train_reduction(tmp_path):
    rows = [('posu_pack_weights_kernel', 1.0), ('conv_igemm_kernel', 1.0), ('bn_apply_kernel', 2.0),
            ('posu_pack_weights_kernel', 4.0), ('conv_igemm_kernel', 8.0), ('wgrad_kernel', 16.0),
            ('multi_tensor_apply_kernel', 32.0)]
    paths = []
    for counter in ('FETCH_SIZE', 'WRITE_SIZE'):
        p = tmp_path / (counter + '.csv')
        with open(p, 'w', newline='') as f:
            w = csv.writer(f)
            w.writerow(['Dispatch_Id', 'Kernel_Name', 'Counter_Name', 'Counter_Value'])
            for i, (n, v) in enumerate(rows):
                w.writerow([i, n, counter, v])
        paths.append(str(p))
    out = subprocess.run([sys.executable, os.path.join(REPO, 'tools', 'pmc_train_traffic.py')] + paths,
                         capture_output=True, text=True, check=True).stdout.splitlines()
    d = json.loads(out[0])
    # the last step starts at the second pack launch: 4 + 8 + 16 + 32 KiB per counter
    assert d['launches'] == 4
    assert d['fetch_bytes_corrected'] == pytest.approx(60 * 1024 * 2)
    assert d['write_bytes'] == pytest.approx(60 * 1024)
    assert d['algorithmic_bytes'] == R.r50_256_train_algorithmic_bytes()
    assert any(ln.startswith('conv wgrad') for ln in out[1:])
