"""posu.optim.Adam (posu_adam_step, ABI 15): the training step's optimizer on the HIP kernel
against torch.optim.Adam, the reference's optimizer (utils/utils.py:79-83)."""
import pytest
import torch

from posu import optim


def test_adam_refuses_cpu_parameters():
    p = torch.nn.Parameter(torch.zeros(8))
    p.grad = torch.ones(8)
    with pytest.raises(RuntimeError, match='MI355X HIP path'):
        optim.Adam([p]).step()


@pytest.mark.gpu
@pytest.mark.parametrize('wd', [0.0, 1e-2])
def test_adam_matches_torch_adam(cuda, wd):
    """Five steps over 150 tensors of ragged sizes (several launches of <= 64 tensors, unaligned
    tails, a tensor without a gradient in one step): parameters and both moments within f32
    rounding of torch.optim.Adam, the step counts equal, state_dict round trip."""
    g = torch.Generator(device=cuda).manual_seed(21)
    sizes = [1, 3, 4, 7, 64, 1000, 2048, 2049, 4096 * 3 + 5, 65536] * 15
    ref = [torch.nn.Parameter(torch.randn(n, device=cuda, generator=g)) for n in sizes]
    ours = [torch.nn.Parameter(p.detach().clone()) for p in ref]
    o_ref = torch.optim.Adam(ref, lr=1e-3, weight_decay=wd, foreach=False)
    o_ours = optim.Adam(ours, lr=1e-3, weight_decay=wd)
    for it in range(5):
        for i, (a, b) in enumerate(zip(ref, ours)):
            if it == 2 and i == 5:
                a.grad = b.grad = None
                continue
            gr = torch.randn(a.shape, device=cuda, generator=g) * (10.0 ** (i % 5 - 2))
            a.grad, b.grad = gr.clone(), gr.clone()
        o_ref.step()
        o_ours.step()
    torch.cuda.synchronize()
    for i, (a, b) in enumerate(zip(ref, ours)):
        torch.testing.assert_close(b, a, rtol=1e-5, atol=1e-7, msg=lambda m: 'param %d: %s' % (i, m))
        for k in ('exp_avg', 'exp_avg_sq'):
            # torch's exp_avg is a lerp, ours beta1 m + (1 - beta1) g: where they nearly cancel the
            # relative difference of two roundings is large, the absolute one is not
            r = o_ref.state[a][k]
            torch.testing.assert_close(o_ours.state[b][k], r, rtol=1e-5, atol=1e-6 * float(r.abs().max()),
                                       msg=lambda m: '%s %d: %s' % (k, i, m))
        assert float(o_ours.state[b]['step']) == float(o_ref.state[a]['step'])
    sd = o_ours.state_dict()
    o2 = optim.Adam(ours, lr=1e-3, weight_decay=wd)
    o2.load_state_dict(sd)
    assert float(o2.state[ours[0]]['step']) == 5.0
