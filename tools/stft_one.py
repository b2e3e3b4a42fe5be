"""Five launches of one spectral kernel at B=512 (for rocprofv3 counter passes).
usage: python tools/stft_one.py [n_fft hop win]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "dl-speech-enhancement_amd")]

import torch  # noqa: E402

from sel import _lib as L  # noqa: E402

n, h, w = (int(v) for v in sys.argv[1:4]) if len(sys.argv) > 3 else (1024, 120, 600)
B, T = 512, 24000
dev = torch.device("cuda")
L.lib()
x = 0.1 * torch.randn(B, T, device=dev)
win = torch.hann_window(w, device=dev)
F, K = 1 + T // h, n // 2 + 1
mag = torch.empty(B, F, K, device=dev)
for _ in range(5):
    L.call("sel_stft_mag_fwd", L.ptr(x), B, T, n, h, w, L.ptr(win), 1e-7, L.ptr(mag), L.stream())
torch.cuda.synchronize()
print("ok", float(mag.mean()))
