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
