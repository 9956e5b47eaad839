"""Data-path kernels against the reference: batch Gaussian
targets vs JointsDatasetCompatible.generate_heatmap and the integral decode of
test_integral.py (tests/golden/datapath.npz, tests/golden/make_datapath_golden.py)."""
import numpy as np
import pytest
import torch

from posu import datapath
from tests.golden.make_datapath_golden import datapath_inputs

pytestmark = pytest.mark.gpu


def test_gaussian_targets_match_reference_generate_heatmap(cuda, golden):
    g = golden('datapath.npz')
    joints, vis, sources, _ = datapath_inputs()
    zero = torch.from_numpy(sources == 'h36m')   # h36m without pseudo labels: weights zeroed
    t, w = datapath.generate_heatmaps(torch.from_numpy(joints).to(cuda), torch.from_numpy(vis).to(cuda),
                                      (256, 256), (64, 64), sigma=2, zero_weight=zero)
    np.testing.assert_array_equal(w.cpu().numpy(), g['weights'])
    np.testing.assert_allclose(t.cpu().numpy(), g['targets'], rtol=1e-6, atol=1e-7)
    assert (t.cpu().numpy() > 0).sum() == (g['targets'] > 0).sum()


def test_integral_decode_matches_reference(cuda, golden):
    g = golden('datapath.npz')
    _, _, _, hm = datapath_inputs()
    out = datapath.integral_preds(torch.from_numpy(hm).to(cuda))
    np.testing.assert_allclose(out.cpu().numpy(), g['integral'], rtol=1e-5, atol=1e-4)
