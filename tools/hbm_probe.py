"""HBM probe: write-only (fill), read-only (sum) and copy bandwidth on large
buffers, to price write-dominated kernels (the STFT |X| kernel writes 4x what it
reads).  usage: python tools/hbm_probe.py   (GPU)"""
import torch


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e-3


def main():
    dev = torch.device("cuda")
    for mb in (256, 1024):
        n = mb * 2**20 // 4
        x = torch.randn(n, device=dev)
        y = torch.empty_like(x)
        t_fill = timed(lambda: y.fill_(1.0))
        t_copy = timed(lambda: y.copy_(x))
        r = torch.empty(1, device=dev)
        t_read = timed(lambda: torch.sum(x, dim=0, out=r))
        B = n * 4
        print(f"{mb} MB: write-only {B / t_fill / 1e9:.0f} GB/s, read-only {B / t_read / 1e9:.0f} GB/s, "
              f"copy {2 * B / t_copy / 1e9:.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
