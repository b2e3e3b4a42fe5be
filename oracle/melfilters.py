"""ORACLE / TEST INFRASTRUCTURE — never imported by the product path.

Restatement of librosa 0.8.1 ``librosa.filters.mel`` (slaney mel scale, slaney
area normalisation, ``htk=False``, ``dtype=float32``), the third-party routine
the reference calls at ``losses/mel_loss.py:54-60``.  librosa is pinned at
``requirements.txt:26`` (``librosa==0.8.1``) and is NOT installed in this
image, so the reference itself is imported for golden generation with this
restatement injected as a stub ``librosa`` module (tests/golden/make_goldens.py).

Parity status: the algorithm below is restated from librosa 0.8.1's published
source (filters.mel / core.convert.{hz_to_mel, mel_to_hz, mel_frequencies,
fft_frequencies}).  No reference test or fixture pins it ("parity unpinned" for
the filterbank constants themselves); everything downstream of the filterbank
is pinned by the goldens.

Numerics follow librosa exactly: ramps are built in float64, each row is
assigned into a float32 array (first rounding), then the float32 array is
multiplied in place by the float64 slaney norm (second rounding).
"""
import numpy as np


def hz_to_mel(frequencies):
    f = np.asanyarray(frequencies, dtype=np.float64)
    f_sp = 200.0 / 3
    mels = f / f_sp
    min_log_hz = 1000.0
    min_log_mel = min_log_hz / f_sp
    logstep = np.log(6.4) / 27.0
    if f.ndim:
        mels = np.array(mels, dtype=np.float64, copy=True)
        log_t = f >= min_log_hz
        mels[log_t] = min_log_mel + np.log(f[log_t] / min_log_hz) / logstep
    elif f >= min_log_hz:
        mels = min_log_mel + np.log(f / min_log_hz) / logstep
    return mels


def mel_to_hz(mels):
    m = np.asanyarray(mels, dtype=np.float64)
    f_sp = 200.0 / 3
    freqs = f_sp * m
    min_log_hz = 1000.0
    min_log_mel = min_log_hz / f_sp
    logstep = np.log(6.4) / 27.0
    if m.ndim:
        freqs = np.array(freqs, dtype=np.float64, copy=True)
        log_t = m >= min_log_mel
        freqs[log_t] = min_log_hz * np.exp(logstep * (m[log_t] - min_log_mel))
    elif m >= min_log_mel:
        freqs = min_log_hz * np.exp(logstep * (m - min_log_mel))
    return freqs


def mel_frequencies(n_mels, fmin, fmax):
    lo = hz_to_mel(fmin)
    hi = hz_to_mel(fmax)
    return mel_to_hz(np.linspace(lo, hi, n_mels))


def mel(sr, n_fft, n_mels=128, fmin=0.0, fmax=None, htk=False, norm="slaney", dtype=np.float32):
    """librosa.filters.mel (0.8.1) -> (n_mels, 1 + n_fft // 2) float32."""
    if htk or norm != "slaney":
        raise NotImplementedError("only the slaney/slaney variant used by the reference")
    if fmax is None:
        fmax = float(sr) / 2
    n_mels = int(n_mels)
    weights = np.zeros((n_mels, int(1 + n_fft // 2)), dtype=dtype)
    fftfreqs = np.linspace(0, float(sr) / 2, int(1 + n_fft // 2), endpoint=True)
    mel_f = mel_frequencies(n_mels + 2, fmin, fmax)
    fdiff = np.diff(mel_f)
    ramps = np.subtract.outer(mel_f, fftfreqs)
    for i in range(n_mels):
        lower = -ramps[i] / fdiff[i]
        upper = ramps[i + 2] / fdiff[i + 1]
        weights[i] = np.maximum(0, np.minimum(lower, upper))
    enorm = 2.0 / (mel_f[2: n_mels + 2] - mel_f[:n_mels])
    weights *= enorm[:, np.newaxis]
    return weights
