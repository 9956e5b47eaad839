"""Cross-view Aggregation (NETWORK.AGGRE, multiview_pose_resnet.py:16-58) on the MI355X
against the reference module's own outputs and gradients (tests/golden/aggregation.npz,
tests/golden/make_aggre_golden.py): the 12 ChannelWiseFC matmuls as one block GEMM."""
import numpy as np
import pytest
import torch

from posu import synthetic as syn
from tests.golden.make_aggre_golden import aggre_inputs

pytestmark = pytest.mark.gpu


def _module(precision, cuda):
    from models.multiview_pose_resnet import Aggregation
    cfg = syn.make_cfg(image_size=64)   # 16 x 16 heatmaps
    agg = Aggregation(cfg, precision=precision).to(cuda)
    views, weights, g = aggre_inputs()
    with torch.no_grad():
        for fc, w in zip(agg.aggre, weights):
            fc.weight.copy_(torch.from_numpy(w))
    return agg, views, g


@pytest.mark.parametrize('precision,tol', [('fp32', 1e-4), ('bf16', 2e-2)])
def test_aggregation_matches_reference_forward_and_backward(cuda, golden, precision, tol):
    gld = golden('aggregation.npz')
    agg, views, g = _module(precision, cuda)
    xs = [torch.from_numpy(v).to(cuda).requires_grad_(True) for v in views]
    out = agg(xs)
    loss = sum((o * torch.from_numpy(gg).to(cuda)).sum() for o, gg in zip(out, g))
    loss.backward()
    got = torch.stack([o.detach() for o in out]).cpu().numpy()
    scale = np.abs(gld['out']).max()
    np.testing.assert_allclose(got, gld['out'], atol=tol * scale, rtol=0)
    dx = torch.stack([x.grad for x in xs]).cpu().numpy()
    np.testing.assert_allclose(dx, gld['dx'], atol=tol * np.abs(gld['dx']).max(), rtol=0)
    norms = np.array([fc.weight.grad.norm().item() for fc in agg.aggre])
    np.testing.assert_allclose(norms, gld['dw_norms'], rtol=max(tol, 1e-4))
    for k, f in (('dw0', 0), ('dw7', 7)):
        ref = gld[k]
        np.testing.assert_allclose(agg.aggre[f].weight.grad.cpu().numpy(), ref, atol=tol * np.abs(ref).max(), rtol=0)


def test_fuse_routing_blends_h36m_samples_only(cuda):
    from core.function import fuse_routing
    r = [torch.randn(3, 16, 8, 8, device=cuda) for _ in range(4)]
    a = [torch.randn(3, 16, 8, 8, device=cuda) for _ in range(4)]
    meta = [{'source': ['h36m', 'mpii', 'h36m']} for _ in range(4)]
    out = fuse_routing(r, a, True, meta)
    for o, rr, aa in zip(out, r, a):
        torch.testing.assert_close(o[0], 3 / 5 * aa[0] + 2 / 5 * rr[0])
        torch.testing.assert_close(o[1], rr[1])
    assert fuse_routing(r, a, False, meta) is r


@pytest.mark.parametrize('precision,tol', [('fp32', 1e-5), ('bf16', 2e-2)])
def test_channel_wise_fc_forward_and_backward_match_matmul(cuda, precision, tol):
    """ChannelWiseFC.forward on its own (multiview_pose_resnet.py:23-28): reshape to
    [N*C, H*W] @ weight, against the same torch ops in fp32 on CPU, with gradients."""
    from models.multiview_pose_resnet import ChannelWiseFC
    g = torch.Generator().manual_seed(3)
    fc = ChannelWiseFC(16 * 16, precision=precision)
    with torch.no_grad():
        fc.weight.copy_(torch.rand(256, 256, generator=g) * 0.1)
    x = torch.randn(3, 16, 16, 16, generator=g)
    gy = torch.randn(3, 16, 16, 16, generator=g)
    xr = x.clone().requires_grad_(True)
    wr = fc.weight.detach().clone().requires_grad_(True)
    ref = torch.matmul(xr.reshape(48, 256), wr).reshape(3, 16, 16, 16)
    (ref * gy).sum().backward()
    fc = fc.to(cuda)
    xd = x.to(cuda).requires_grad_(True)
    out = fc(xd)
    (out * gy.to(cuda)).sum().backward()
    s = ref.abs().max().item()
    np.testing.assert_allclose(out.detach().cpu().numpy(), ref.detach().numpy(), atol=tol * s, rtol=0)
    np.testing.assert_allclose(xd.grad.cpu().numpy(), xr.grad.numpy(), atol=tol * xr.grad.abs().max().item(), rtol=0)
    np.testing.assert_allclose(fc.weight.grad.cpu().numpy(), wr.grad.numpy(), atol=tol * wr.grad.abs().max().item(),
                               rtol=0)
