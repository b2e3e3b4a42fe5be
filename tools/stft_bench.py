"""Microbenchmark of the spectral kernels at SURVEY §8d's HBM-measurement size
(B >= 512 signals x 1 s @ 24 kHz, beyond the 256 MB Infinity Cache).

Per signal per resolution: STFT magnitude bytes = 4*(T + F*K)
(read the waveform once, write the magnitudes once), flops = F*(2.5 n log2 n + n + 4K).
usage: python tools/stft_bench.py [B]     (GPU)
"""
import math
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "dl-speech-enhancement_amd")]

import torch  # noqa: E402

from sel import _lib as L  # noqa: E402
from sel import spectral as S  # noqa: E402

RES = [(1024, 120, 600), (2048, 240, 1200), (512, 50, 240), (2048, 300, 2048)]


def timed(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e-3


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    T = 24000
    dev = torch.device("cuda")
    L.lib()
    x = 0.1 * torch.randn(B, T, device=dev)
    y = 0.1 * torch.randn(B, T, device=dev)
    print(f"B={B} T={T}")
    # measured HBM peak: device-to-device copy of 2 GiB (read + write bytes)
    src = torch.empty(2 ** 29, device=dev)
    dst = torch.empty_like(src)
    sc = timed(lambda: dst.copy_(src), iters=10)
    print(f"measured copy bandwidth: {2 * src.numel() * 4 / sc / 1e9:.0f} GB/s (2 GiB D2D copy)")
    del src, dst
    print("| kernel | n_fft/hop/win | us | alg. bytes | GB/s | % of 8 TB/s | GFLOP/s |")
    print("|---|---|---|---|---|---|---|")
    for n, h, w in RES:
        win = torch.hann_window(w, device=dev)
        F, K = 1 + T // h, n // 2 + 1
        nbytes = 4 * B * (T + F * K)
        flops = B * F * (2.5 * n * math.log2(n) + n + 4 * K)
        mag = torch.empty(B, F, K, device=dev)
        s = timed(lambda: L.call("sel_stft_mag_fwd", L.ptr(x), B, T, n, h, w, L.ptr(win), 1e-7, L.ptr(mag),
                                 L.stream()))
        print(f"| stft_mag_fwd | {n}/{h}/{w} | {s * 1e6:.1f} | {nbytes / 1e6:.1f} MB | {nbytes / s / 1e9:.0f} | "
              f"{100 * nbytes / s / 8e12:.1f} | {flops / s / 1e9:.0f} |", flush=True)
        # fused STFT loss forward: both signals, partial sums only (compute-bound)
        xr = x.clone().requires_grad_(True)

        def fused():
            return S.StftLoss.apply(xr, y, n, h, w, win) if hasattr(S, "StftLoss") else None
        try:
            s2 = timed(lambda: fused())
            print(f"| stft_loss_fwd (x,y) | {n}/{h}/{w} | {s2 * 1e6:.1f} | {2 * 4 * B * T / 1e6:.1f} MB in | "
                  f"{2 * 4 * B * T / s2 / 1e9:.0f} | - | {2 * flops / s2 / 1e9:.0f} |", flush=True)
        except Exception as e:  # noqa: BLE001
            print(f"| stft_loss_fwd | {n}/{h}/{w} | n/a ({str(e)[:60]}) |")
        # magnitude backward (the kernel alone: slab + overlap-add) given dL/d|X|
        gm = torch.randn(B, F, K, device=dev)
        gx = torch.empty_like(x)
        ws = torch.empty(lib_ws(B, T, n, h, w), dtype=torch.uint8, device=dev)
        s3 = timed(lambda: L.call("sel_stft_mag_bwd", L.ptr(x), B, T, n, h, w, L.ptr(win), 1e-7, L.ptr(gm),
                                  L.ptr(gx), L.ptr(ws), ws.numel(), L.stream()))
        print(f"| stft_mag_bwd | {n}/{h}/{w} | {s3 * 1e6:.1f} | - | - | - | {flops / s3 / 1e9:.0f} |", flush=True)
    # the C3 mel loss: 45 * L1(logmel(y_hat), logmel(y)), 2048/300/2048, fwd + bwd at B=64
    from losses import MultiMelSpectrogramLoss
    ml = MultiMelSpectrogramLoss(fs=24000, fft_sizes=[2048], hop_sizes=[300], win_lengths=[None],
                                 num_mels=80, fmin=0, fmax=12000, log_base=None).to(dev)
    yh = (0.1 * torch.randn(64, 1, T, device=dev)).requires_grad_(True)
    yc = 0.1 * torch.randn(64, 1, T, device=dev)

    def mel_step():
        ml(yh, yc).backward()
    s4 = timed(mel_step)
    print(f"| mel loss fwd+bwd (B=64) | 2048/300/2048 | {s4 * 1e6:.1f} | - | - | - | - |", flush=True)


def lib_ws(B, T, n, h, w):
    return int(L.lib().sel_stft_bwd_workspace(B, T, n, h, w))


if __name__ == "__main__":
    main()
