"""HBM ceiling of the layer1 Bottleneck tail's traffic shape, for comparison with the conv:
bf16 NHWC [128, 64, 64, 256] tensors (268 MB each): copy (read 1 + write 1) and
residual add (read 2 + write 1), timed with HIP events (min over rounds)."""
import torch


def timeit(fn, reps=20, rounds=3):
    best = 1e9
    for _ in range(rounds):
        fn()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        b.synchronize()
        best = min(best, a.elapsed_time(b) / reps)
    return best * 1e3


def main():
    dev = torch.device('cuda', 0)
    x = torch.randn(128, 64, 64, 256, device=dev).to(torch.bfloat16)
    r = torch.randn_like(x)
    y = torch.empty_like(x)
    nb = x.numel() * 2
    t = timeit(lambda: y.copy_(x))
    print('copy      %7.1f us  %5.2f TB/s' % (t, 2 * nb / t / 1e6))
    t = timeit(lambda: torch.add(x, r, out=y))
    print('add       %7.1f us  %5.2f TB/s' % (t, 3 * nb / t / 1e6))
    x64 = torch.randn(128, 64, 64, 64, device=dev).to(torch.bfloat16)
    t = timeit(lambda: torch.add(r, x64.repeat(1, 1, 1, 4), out=y))
    print('read 64ch + res + write (with repeat) %7.1f us' % t)


if __name__ == '__main__':
    main()
