"""STFT-based loss modules — drop-in for the reference ``losses/stft_loss.py``.

Same names, constructor arguments, buffers and return values as the reference
(stft :19-35, SpectralConvergenceLoss :38-56, LogSTFTMagnitudeLoss :59-77,
STFTLoss :80-117, MultiResolutionSTFTLoss :120-170); the arithmetic runs in the
HIP kernels of libsel.so (sel/spectral.py).  ``STFTLoss.forward`` uses the fused
per-frame kernel that never materialises the magnitudes.
"""
import torch

from sel import spectral as S


def stft(x, fft_size, hop_size, win_length, window, eps=1e-7):
    """|STFT| (B, #frames, fft_size // 2 + 1) — reference stft_loss.py:19-35."""
    return S.stft_mag(x, fft_size, hop_size, win_length, window, eps)


class SpectralConvergenceLoss(torch.nn.Module):
    """||y - x||_F / ||y||_F over the whole tensor (stft_loss.py:38-56)."""

    def forward(self, x_mag, y_mag):
        return S.MagPairLoss.apply(x_mag, y_mag)[0]


class LogSTFTMagnitudeLoss(torch.nn.Module):
    """mean |ln y - ln x| (stft_loss.py:59-77)."""

    def forward(self, x_mag, y_mag):
        return S.MagPairLoss.apply(x_mag, y_mag)[1]


class STFTLoss(torch.nn.Module):
    """STFT loss module (stft_loss.py:80-117)."""

    def __init__(self, fft_size=1024, hop_size=120, win_length=600, window="hann_window"):
        super().__init__()
        self.fft_size = fft_size
        self.hop_size = hop_size
        self.win_length = win_length
        self.spectral_convergence_loss = SpectralConvergenceLoss()
        self.log_stft_magnitude_loss = LogSTFTMagnitudeLoss()
        self.register_buffer("window", getattr(torch, window)(win_length))

    def forward(self, x, y):
        if y.requires_grad:  # reference differentiates both; fused kernel only w.r.t. x
            x_mag = stft(x, self.fft_size, self.hop_size, self.win_length, self.window)
            y_mag = stft(y, self.fft_size, self.hop_size, self.win_length, self.window)
            out = S.MagPairLoss.apply(x_mag, y_mag)
            return out[0], out[1]
        return S.stft_loss(x, y, self.fft_size, self.hop_size, self.win_length, self.window)


class MultiResolutionSTFTLoss(torch.nn.Module):
    """Multi resolution STFT loss module (stft_loss.py:120-170)."""

    def __init__(self, fft_sizes=[1024, 2048, 512], hop_sizes=[120, 240, 50],
                 win_lengths=[600, 1200, 240], window="hann_window"):
        super().__init__()
        assert len(fft_sizes) == len(hop_sizes) == len(win_lengths)
        self.stft_losses = torch.nn.ModuleList()
        for fft_size, hop_size, win_length in zip(fft_sizes, hop_sizes, win_lengths):
            self.stft_losses += [STFTLoss(fft_size, hop_size, win_length, window)]

    def forward(self, x, y):
        if len(x.shape) == 3:
            x = x.view(-1, x.size(2))
            y = y.view(-1, y.size(2))
        sc_loss = 0.0
        mag_loss = 0.0
        for f in self.stft_losses:
            sc_l, mag_l = f(x, y)
            sc_loss = sc_loss + sc_l
            mag_loss = mag_loss + mag_l
        n = len(self.stft_losses)
        return sc_loss / n, mag_loss / n
