"""Mel-spectrogram loss modules — drop-in for the reference ``losses/mel_loss.py``.

MelSpectrogram (:19-94) and MultiMelSpectrogramLoss (:97-155) keep the
reference's constructor arguments and buffers (``window``, ``melmat``; same
state_dict keys).  The slaney filterbank that the reference takes from
librosa 0.8.1 is built by sel/melbank.py.  ``center``/``normalized``/``onesided``
are stored but — exactly as in the reference — not used (torch.stft defaults).
"""
import torch
import torch.nn.functional as F

from sel import spectral as S
from sel.melbank import slaney_mel


class MelSpectrogram(torch.nn.Module):
    """Calculate Mel-spectrogram (mel_loss.py:19-94)."""

    def __init__(self, fs=22050, fft_size=1024, hop_size=256, win_length=None,
                 window="hann_window", num_mels=80, fmin=80, fmax=7600, center=True,
                 normalized=False, onesided=True, eps=1e-10, log_base=10.0):
        super().__init__()
        self.fft_size = fft_size
        self.hop_size = hop_size
        self.win_length = win_length if win_length is not None else fft_size
        self.center = center
        self.normalized = normalized
        self.onesided = onesided
        self.register_buffer("window", getattr(torch, window)(self.win_length))
        self.eps = eps
        fmin = 0 if fmin is None else fmin
        fmax = fs / 2 if fmax is None else fmax
        melmat = slaney_mel(sr=fs, n_fft=fft_size, n_mels=num_mels, fmin=fmin, fmax=fmax)
        self.register_buffer("melmat", torch.from_numpy(melmat.T).float())
        self.log_base = log_base
        if log_base not in S.LOG_KIND:
            raise ValueError(f"log_base: {log_base} is not supported.")
        self._log_kind = S.LOG_KIND[log_base]
        self._ranges_cache = {}

    def _ranges(self):
        mm = self.melmat
        key = (mm.device, mm.data_ptr(), mm._version)
        hit = self._ranges_cache.get("key")
        if hit != key:
            kr, mr = S.mel_ranges(mm)
            self._ranges_cache = {"key": key, "kr": kr.to(mm.device), "mr": mr.to(mm.device)}
        return self._ranges_cache["kr"], self._ranges_cache["mr"]

    def _args(self):
        kr, mr = self._ranges()
        return (self.fft_size, self.hop_size, self.win_length, self.window.contiguous(),
                self.melmat.contiguous(), kr, mr, float(self.eps), self._log_kind)

    def forward(self, x):
        """(B, T) or (B, C, T) -> log-mel (B, #mels, #frames)."""
        return S.LogMel.apply(S._signal_2d(x), *self._args())

    def l1(self, y_hat, y):
        """Fused mean |mel(y_hat) - mel(y)| (the body of MultiMelSpectrogramLoss)."""
        if y.requires_grad:
            return F.l1_loss(self(y_hat), self(y))
        return S.MelL1.apply(S._signal_2d(y_hat), S._signal_2d(y).detach(), *self._args())


class MultiMelSpectrogramLoss(torch.nn.Module):
    """Multi resolution Mel-spectrogram loss (mel_loss.py:97-155)."""

    def __init__(self, fs=22050, fft_sizes=[1024, 2048, 512], hop_sizes=[120, 240, 50],
                 win_lengths=[600, 1200, 240], window="hann_window", num_mels=80, fmin=80,
                 fmax=7600, center=True, normalized=False, onesided=True, eps=1e-10,
                 log_base=10.0):
        super().__init__()
        assert len(fft_sizes) == len(hop_sizes) == len(win_lengths)
        self.mel_transfers = torch.nn.ModuleList()
        for fft_size, hop_size, win_length in zip(fft_sizes, hop_sizes, win_lengths):
            self.mel_transfers += [
                MelSpectrogram(fs=fs, fft_size=fft_size, hop_size=hop_size, win_length=win_length,
                               window=window, num_mels=num_mels, fmin=fmin, fmax=fmax,
                               center=center, normalized=normalized, onesided=onesided, eps=eps,
                               log_base=log_base)
            ]

    def forward(self, y_hat, y):
        mel_loss = None
        for f in self.mel_transfers:
            l = f.l1(y_hat, y)
            mel_loss = l if mel_loss is None else mel_loss + l
        if len(self.mel_transfers) > 1:
            mel_loss = mel_loss / len(self.mel_transfers)
        return mel_loss
