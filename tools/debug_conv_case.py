"""Debug helper: run one conv case on the GPU against torch and summarise where it differs."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'pose-unsupervised_amd', 'lib'), REPO, os.path.join(REPO, 'tests')]
import torch  # noqa: E402

from test_gpu_kernels import _conv_case  # noqa: E402
from posu import ops  # noqa: E402
from posu._native import F32, BF16  # noqa: E402


def main():
    cuda = torch.device('cuda', 0)
    for n in (8, 16, 32, 64):
        for cfg in (-1, 3, 5):
            ops.force_conv_config(cfg)
            case = (n, 64, 32, 32, 256, 3, 1, 1, True, True)
            got, ref = _conv_case(cuda, F32, *case)
            bad = (got - ref).abs() > 1e-3
            frac = bad.float().mean().item()
            per_img = bad.float().mean(dim=(1, 2, 3))
            print('n=%d cfg=%d bad=%.4f first bad imgs %s rows %s' % (
                n, cfg, frac, torch.nonzero(per_img > 0).flatten()[:8].tolist(),
                torch.nonzero(bad.float().mean(dim=(0, 1, 3)) > 0).flatten()[:8].tolist()), flush=True)
    ops.force_conv_config(-1)


if __name__ == '__main__':
    main()
