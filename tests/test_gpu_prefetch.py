"""The side-stream weight prefetch (posu_prefetch, plan.PREFETCH): the kernel over ragged sizes and
its refusals, and a PoseResNet-50 forward bit-identical with and without it, eager and captured
in a hipGraph (the side stream joins the capture)."""
import pytest
import torch

from posu import ops
from posu import plan as P
from posu import synthetic as syn

pytestmark = pytest.mark.gpu


def test_prefetch_sizes_and_refusals(cuda):
    buf = torch.arange(1 << 20, device=cuda, dtype=torch.int32)
    ref = buf.clone()
    for nbytes in (4, 60, 64, 68, 1000, 4096, (1 << 22) - 4, 1 << 22):
        for wg in (0, 1, 7, 32):
            ops.prefetch(buf.view(torch.uint8)[:nbytes], wg)
    ops.prefetch(buf[:0])   # empty: no launch
    torch.cuda.synchronize()
    assert torch.equal(buf, ref)   # nothing written
    with pytest.raises(RuntimeError, match='16-byte aligned'):
        ops.prefetch(buf[1:])
    with pytest.raises(RuntimeError, match='under 4 bytes'):
        ops.prefetch(buf.view(torch.uint8)[:2])
    with pytest.raises(RuntimeError, match='negative'):
        ops.prefetch(buf, -1)


def _net(cuda):
    from models.pose_resnet import get_pose_net
    net = get_pose_net(syn.make_cfg(num_layers=50, image_size=256), is_train=False, precision='bf16')
    net.load_state_dict(syn.synthetic_state_dict(net.state_dict(), seed=1, bn_stats=syn.load_bn_stats(50, 256)))
    return net.to(cuda).eval()


@pytest.mark.parametrize('chunks', [1, 2])
def test_prefetch_forward_bit_identical_eager_and_graph(cuda, chunks):
    net = _net(cuda)
    views = [v.to(cuda) for v in syn.synthetic_views(4, 2, 256, seed=5)]
    saved = P.PREFETCH
    try:
        with torch.no_grad():
            plan = net.plan(cuda)
            P.PREFETCH = False
            hm0 = plan.run(plan.pack_input(views), chunks=chunks)[0]
            P.PREFETCH = True
            hm1 = plan.run(plan.pack_input(views), chunks=chunks)[0]
            torch.cuda.synchronize()
            assert not P._Prefetch.pending   # joined at the end of run()
            assert P._Prefetch.streams       # and it did issue prefetches
            assert torch.equal(hm0, hm1)
            s = torch.cuda.Stream(cuda)
            s.wait_stream(torch.cuda.current_stream(cuda))
            with torch.cuda.stream(s):
                plan.run(plan.pack_input(views), chunks=chunks)
            torch.cuda.current_stream(cuda).wait_stream(s)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                hmg = plan.run(plan.pack_input(views), chunks=chunks)[0]
            g.replay()
            torch.cuda.synchronize()
            assert torch.equal(hmg, hm0)
    finally:
        P.PREFETCH = saved
