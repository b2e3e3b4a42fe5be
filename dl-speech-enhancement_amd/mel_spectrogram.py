"""mel_spectrogram.py drop-in: the eval Mel-L1 metric (reference :38-44).

The reference builds ``mel_spectrogram = torchaudio.transforms.MelSpectrogram(48000)``
and ``Mel_L1(pred, target) = L1(mel(pred), mel(target))``; its remaining
module-level code (soundfile I/O, plots, printing every torchmetrics measure,
:46-118) is not part of the hot path and is not reproduced.

``MelSpectrogram`` mirrors torchaudio's transform signature and defaults
(n_fft 400, hop = win // 2, periodic Hann, center/reflect, onesided, power 2,
HTK mel scale, no norm) and runs the sel_power_mel_fwd HIP kernel (mixed-radix
FFT for n_fft = 400).  Only the defaults' feature set is implemented: other
options raise instead of silently differing.
"""
import torch
from torch import nn

from sel import spectral as S
from sel.melbank import htk_fbanks


class MelSpectrogram(nn.Module):
    """torchaudio.transforms.MelSpectrogram (2.1.1) on the MI355X path."""

    def __init__(self, sample_rate=16000, n_fft=400, win_length=None, hop_length=None, f_min=0.0, f_max=None,
                 pad=0, n_mels=128, window_fn=torch.hann_window, power=2.0, normalized=False, wkwargs=None,
                 center=True, pad_mode="reflect", onesided=None, norm=None, mel_scale="htk"):
        super().__init__()
        unsupported = {"pad": pad != 0, "normalized": bool(normalized), "center": not center,
                       "pad_mode": pad_mode != "reflect", "onesided": onesided is False, "norm": norm is not None,
                       "mel_scale": mel_scale != "htk", "power": power is None}
        bad = [k for k, v in unsupported.items() if v]
        if bad:
            raise NotImplementedError(f"sel MelSpectrogram: options {bad} differ from the reference's defaults")
        self.sample_rate = sample_rate
        self.n_fft = n_fft
        self.win_length = win_length if win_length is not None else n_fft
        self.hop_length = hop_length if hop_length is not None else self.win_length // 2
        self.power = float(power)
        self.n_mels = n_mels
        self.f_min = f_min
        self.f_max = f_max if f_max is not None else float(sample_rate // 2)
        window = window_fn(self.win_length) if wkwargs is None else window_fn(self.win_length, **wkwargs)
        self.register_buffer("window", window.float())
        fb = htk_fbanks(n_fft // 2 + 1, float(f_min), self.f_max, n_mels, sample_rate)
        self.register_buffer("fb", fb)
        kr, _ = S.mel_ranges(fb)
        self.register_buffer("krange", kr, persistent=False)

    def forward(self, waveform):
        shape = waveform.shape
        x = waveform.reshape(-1, shape[-1]).float()
        out = S.power_mel(x, self.n_fft, self.hop_length, self.win_length, self.window, self.fb, self.krange,
                          self.power)
        return out.reshape(shape[:-1] + out.shape[-2:])


mel_spectrogram = MelSpectrogram(48000)
mae = nn.L1Loss()


def Mel_L1(pred, target):
    """reference :40-44; the module buffers follow the input's device."""
    if mel_spectrogram.window.device != pred.device:
        mel_spectrogram.to(pred.device)
    with torch.no_grad():
        return mae(mel_spectrogram(pred), mel_spectrogram(target))
