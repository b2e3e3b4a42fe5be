"""Slaney mel filterbank, constructor-time parameter (host numpy).

Replaces the reference's call ``librosa.filters.mel(sr, n_fft, n_mels, fmin, fmax)``
(losses/mel_loss.py:54-60; librosa==0.8.1, requirements.txt:26 — not installed
in this image).  librosa 0.8.1 semantics: slaney mel scale (linear below 1 kHz,
log above), triangular ramps built in float64, each row rounded into a float32
array, then multiplied in place by the float64 slaney area norm (second
rounding).  Returns (n_mels, 1 + n_fft // 2) float32 like librosa; the module
stores its transpose as the ``melmat`` buffer exactly as the reference does.
"""
import numpy as np

_F_SP = 200.0 / 3
_MIN_LOG_HZ = 1000.0
_MIN_LOG_MEL = _MIN_LOG_HZ / _F_SP
_LOGSTEP = np.log(6.4) / 27.0


def _hz_to_mel(f):
    f = np.atleast_1d(np.asarray(f, dtype=np.float64))
    m = f / _F_SP
    hi = f >= _MIN_LOG_HZ
    m[hi] = _MIN_LOG_MEL + np.log(f[hi] / _MIN_LOG_HZ) / _LOGSTEP
    return m


def _mel_to_hz(m):
    m = np.atleast_1d(np.asarray(m, dtype=np.float64))
    f = _F_SP * m
    hi = m >= _MIN_LOG_MEL
    f[hi] = _MIN_LOG_HZ * np.exp(_LOGSTEP * (m[hi] - _MIN_LOG_MEL))
    return f


def slaney_mel(sr, n_fft, n_mels=128, fmin=0.0, fmax=None):
    if fmax is None:
        fmax = float(sr) / 2
    n_bins = int(1 + n_fft // 2)
    fft_hz = np.linspace(0, float(sr) / 2, n_bins, endpoint=True)
    edges = _mel_to_hz(np.linspace(_hz_to_mel(fmin)[0], _hz_to_mel(fmax)[0], int(n_mels) + 2))
    widths = np.diff(edges)
    ramps = edges[:, None] - fft_hz[None, :]
    w = np.zeros((int(n_mels), n_bins), dtype=np.float32)
    for i in range(int(n_mels)):
        rise = -ramps[i] / widths[i]
        fall = ramps[i + 2] / widths[i + 1]
        w[i] = np.maximum(0, np.minimum(rise, fall))
    w *= (2.0 / (edges[2:int(n_mels) + 2] - edges[:int(n_mels)]))[:, None]
    return w


def htk_fbanks(n_freqs, f_min, f_max, n_mels, sample_rate):
    """torchaudio.functional.melscale_fbanks(..., norm=None, mel_scale="htk")
    (torchaudio 2.1.1, the default of transforms.MelSpectrogram used by
    mel_spectrogram.py:38; torchaudio is not installed here).  fp32 like
    torchaudio: linspace bin freqs, HTK mel points, min(down, up) triangles.
    Returns (n_freqs, n_mels) float32 — torchaudio's `fb` buffer layout."""
    import torch
    all_freqs = torch.linspace(0, sample_rate // 2, n_freqs)
    m_min = 2595.0 * np.log10(1.0 + f_min / 700.0)
    m_max = 2595.0 * np.log10(1.0 + f_max / 700.0)
    m_pts = torch.linspace(float(m_min), float(m_max), n_mels + 2)
    f_pts = 700.0 * (10.0 ** (m_pts / 2595.0) - 1.0)
    f_diff = f_pts[1:] - f_pts[:-1]
    slopes = f_pts.unsqueeze(0) - all_freqs.unsqueeze(1)
    down = (-1.0 * slopes[:, :-2]) / f_diff[:-1]
    up = slopes[:, 2:] / f_diff[1:]
    return torch.max(torch.zeros(1), torch.min(down, up))
