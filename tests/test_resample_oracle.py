"""CPU checks of the resampling oracle (oracle/ref_ops.resample, a restatement of
torchaudio 2.1.1 functional.resample / sinc_interp_hann, which is absent here:
parity unpinned by any reference fixture).  Properties only: output length
ceil(len * new / orig) on the reduced ratio, pass-band sinusoids kept, a
down/up round trip of band-limited content, agreement with an independent
polyphase resampler (scipy.signal.resample_poly) in the pass band."""
import math

import numpy as np
import pytest
import torch

from oracle import ref_ops as R


@pytest.mark.parametrize("orig,new,n", [(48000, 24000, 9601), (16000, 24000, 4000), (44100, 24000, 8821),
                                        (24000, 48000, 3000), (22050, 24000, 2205)])
def test_length_and_passband_sine(orig, new, n):
    t = torch.arange(n, dtype=torch.float64) / orig
    x = torch.sin(2 * math.pi * 1000.0 * t).float().view(1, 1, -1)
    y = R.resample(x, orig, new)
    g = math.gcd(orig, new)
    assert y.shape[-1] == math.ceil((new // g) * n / (orig // g))
    ty = torch.arange(y.shape[-1], dtype=torch.float64) / new
    ref = torch.sin(2 * math.pi * 1000.0 * ty)
    m = 200  # away from the zero-padded ends
    err = (y[0, 0, m:-m].double() - ref[m:-m]).abs().max().item()
    assert err < 2e-3, err


def test_round_trip_band_limited():
    rng = np.random.default_rng(0)
    x = torch.zeros(2, 24000, dtype=torch.float64)
    t = torch.arange(24000, dtype=torch.float64) / 24000
    for f in rng.uniform(50, 8000, 12):
        x += torch.sin(2 * math.pi * f * t + rng.uniform(0, 6.28))
    up = R.resample(x.float(), 24000, 48000)
    back = R.resample(up, 48000, 24000)
    err = (back[:, 500:-500].double() - x[:, 500:-500]).abs().max().item() / x.abs().max().item()
    assert err < 1e-2, err


def test_matches_scipy_polyphase_in_passband():
    from scipy.signal import resample_poly
    rng = np.random.default_rng(1)
    t = np.arange(48000) / 48000
    x = sum(np.sin(2 * np.pi * f * t + p) for f, p in zip(rng.uniform(50, 9000, 10), rng.uniform(0, 6.28, 10)))
    y = R.resample(torch.from_numpy(x).float().view(1, -1), 48000, 24000)[0].double().numpy()
    ys = resample_poly(x, 1, 2)
    err = np.abs(y[300:-300] - ys[300:-300]).max() / np.abs(x).max()
    assert err < 1e-2, err
