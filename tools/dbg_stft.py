"""Locate STFT-magnitude mismatches (frames / bins) against the oracle (GPU debug aid)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "dl-speech-enhancement_amd")]

import torch  # noqa: E402

from oracle import ref_ops as R  # noqa: E402
from sel import spectral as S  # noqa: E402

for (n, h, w) in [(1024, 120, 600), (512, 50, 240)]:
    g = torch.Generator().manual_seed(1)
    x = 0.1 * torch.randn(2, 24000, generator=g)
    ref = R.stft_mag(x.double(), n, h, w, R.hann(w).double()).float()
    out = S.stft_mag(x.cuda(), n, h, w, torch.hann_window(w).cuda()).cpu()
    err = (out - ref).abs() / ref.abs().mean()
    print(n, "rel", ((out - ref).norm() / ref.norm()).item())
    bad = (err > 1e-3).nonzero()
    print("nbad", bad.shape[0], "of", err.numel())
    print("bad frames", sorted(set(bad[:, 1].tolist()))[:40])
    print("bad bins", sorted(set(bad[:, 2].tolist()))[:60])
