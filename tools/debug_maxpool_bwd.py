import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'pose-unsupervised_amd', 'lib'))
import torch, torch.nn.functional as F
from posu import ops, train_ops as T
from posu._native import BF16, F32
cuda = torch.device('cuda')
g = torch.Generator().manual_seed(16)
x = torch.randint(-2, 3, (2, 64, 17, 16), generator=g).float().requires_grad_(True)
y = F.max_pool2d(x, 3, stride=2, padding=1)
gy = torch.randint(-4, 5, y.shape, generator=g).float()
(gx_ref,) = torch.autograd.grad(y, x, gy)
for code in (F32, BF16):
    dt = ops.torch_dtype(code)
    xd = x.detach().permute(0, 2, 3, 1).contiguous().to(cuda, dt)
    gx = T.maxpool3x3s2_bwd(xd, gy.permute(0, 2, 3, 1).contiguous().to(cuda, dt))
    idx = T._WS[(str(xd.device), 'maxpool')][: 2 * 9 * 8 * 64].view(2, 9, 8, 64).cpu()
    got = gx.float().cpu().permute(0, 3, 1, 2)
    bad = (got != gx_ref).nonzero()
    print('code', code, 'mismatches', len(bad))
    for b in bad[:6].tolist():
        n, c, h, w = b
        print(' at', b, 'got', got[n, c, h, w].item(), 'ref', gx_ref[n, c, h, w].item())
        for oy in range(max(0, (h - 1) // 2), min(9, (h + 1) // 2 + 1)):
            for ox in range(max(0, (w - 1) // 2), min(8, (w + 1) // 2 + 1)):
                win = x.detach()[n, c, max(0, 2*oy-1):2*oy+2, max(0, 2*ox-1):2*ox+2]
                print('   win', oy, ox, win.tolist(), 'idx', idx[n, oy, ox, c].item(), 'gy', gy[n, c, oy, ox].item())
