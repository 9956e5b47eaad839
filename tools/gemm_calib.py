"""Calibration: torch.matmul (hipBLASLt) bf16 on the GEMM shapes of the R50@256 convs at
batch 128 (M = output pixels, K = window taps x Cin, N = Cout).  Not part of the product:
it tells what a tuned library GEMM reaches on the same shapes on this GPU, as a yardstick
for the implicit-GEMM conv kernels (run on the GPU box)."""
import torch

SHAPES = [
    ('square 8192', 8192, 8192, 8192),
    ('l2 conv1 (s1 1x1 512->128)', 131072, 512, 128),
    ('l2 conv2 (3x3 128)', 131072, 1152, 128),
    ('l3 conv1 (1x1 1024->256)', 32768, 1024, 256),
    ('l3 conv2 (3x3 256)', 32768, 2304, 256),
    ('l3 conv3 (1x1 256->1024)', 32768, 256, 1024),
    ('l4 conv1 (1x1 2048->512)', 8192, 2048, 512),
    ('l4 conv2 (3x3 512)', 8192, 4608, 512),
    ('l4 conv3 (1x1 512->2048)', 8192, 512, 2048),
    ('deconv1 (per parity 2048x4)', 32768, 8192, 256),
    ('deconv3 (per parity 256x4)', 524288, 1024, 256),
]


def main():
    torch.manual_seed(0)
    dev = torch.device('cuda', 0)
    for name, m, k, n in SHAPES:
        a = torch.randn(m, k, device=dev, dtype=torch.bfloat16)
        b = torch.randn(k, n, device=dev, dtype=torch.bfloat16)
        for _ in range(5):
            c = a @ b
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 20
        e0.record()
        for _ in range(reps):
            c = a @ b
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1000 / reps
        print('%-32s M %7d K %5d N %5d  %8.1f us  %7.1f TFLOP/s' % (name, m, k, n, us, 2.0 * m * n * k / us / 1e6),
              flush=True)
        del a, b, c


if __name__ == '__main__':
    main()
