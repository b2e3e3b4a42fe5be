"""Per-launch times of the STFT |X| probe (bench.stft_kernel_roofline's kernel
and shape) over many back-to-back launches, to see whether the rate drifts
with sustained load (clock / power), next to the copy probe's."""
import sys
import torch
sys.path.insert(0, "dl-speech-enhancement_amd")
sys.path.insert(0, ".")
from sel import _lib as L  # noqa: E402

dev = torch.device("cuda")
B, T, n, h, w = 2048, 24000, 1024, 120, 600
F, K = 1 + T // h, n // 2 + 1
x = 0.1 * torch.randn(B, T, device=dev)
win = torch.hann_window(w, device=dev)
mag = torch.empty(B, F, K, device=dev)
src = torch.empty(2 ** 28, device=dev)
dst = torch.empty_like(src)
cus = torch.cuda.get_device_properties(dev).multi_processor_count


def trace(fn, iters):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    for e0, e1 in ev:
        e0.record()
        fn()
        e1.record()
    torch.cuda.synchronize()
    return [round(e0.elapsed_time(e1) * 1e3, 1) for e0, e1 in ev]


stft = lambda: L.call("sel_stft_mag_fwd", L.ptr(x), B, T, n, h, w, L.ptr(win), 1e-7, L.ptr(mag), L.stream())
copy = lambda: L.call("sel_probe_copy_f4", L.ptr(src), L.ptr(dst), src.numel() // 4, 8 * cus, L.stream())
print("copy us", trace(copy, 10))
print("stft us", trace(stft, 40))
torch.cuda.synchronize()
import time  # noqa: E402
time.sleep(2.0)
print("stft us after 2 s idle", trace(stft, 10))
print("copy us", trace(copy, 10))
