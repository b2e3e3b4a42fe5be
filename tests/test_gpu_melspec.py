"""a8: mel_spectrogram.py's eval power-mel (torchaudio MelSpectrogram(48000) defaults)
and Mel_L1, against the oracle restatement.  torchaudio is absent here, so parity
is unpinned beyond that restatement.

Tolerance: 1e-4 norm-wise relative on the power-mel (power 2 doubles the FFT's
relative error; the mixed-radix FFT is fp32 like torch's), 1e-4 on Mel_L1."""
import pytest
import torch

from oracle import ref_ops as R

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / b.norm()).item()


@pytest.mark.parametrize("shape", [(2, 48000), (1, 2, 12345), (3, 401)])
def test_power_mel_default_vs_oracle(gpu, shape):
    from mel_spectrogram import MelSpectrogram
    torch.manual_seed(sum(shape))
    x = 0.1 * torch.randn(*shape)
    m = MelSpectrogram(48000).to(gpu)
    out = m(x.to(gpu))
    ref = R.power_melspec(x, sample_rate=48000)
    assert out.shape == ref.shape
    assert _rel(out, ref) < 1e-4


@pytest.mark.parametrize("sr,n_fft,hop,win,n_mels", [(24000, 240, 60, 240, 40), (16000, 512, 128, 400, 80),
                                                      (22050, 300, 75, 300, 64), (48000, 1024, 256, 1024, 128)])
def test_power_mel_other_sizes_vs_oracle(gpu, sr, n_fft, hop, win, n_mels):
    from mel_spectrogram import MelSpectrogram
    torch.manual_seed(n_fft)
    x = 0.1 * torch.randn(2, 8000)
    m = MelSpectrogram(sr, n_fft=n_fft, hop_length=hop, win_length=win, n_mels=n_mels).to(gpu)
    out = m(x.to(gpu))
    ref = R.power_melspec(x, sample_rate=sr, n_fft=n_fft, hop_length=hop, win_length=win, n_mels=n_mels)
    assert _rel(out, ref) < 1e-4


def test_mel_l1_vs_oracle(gpu):
    import mel_spectrogram as MS
    torch.manual_seed(1)
    t = 0.1 * torch.randn(1, 48000)
    p = t + 0.02 * torch.randn(1, 48000)
    v = MS.Mel_L1(p.to(gpu), t.to(gpu))
    r = R.mel_l1(p, t, sample_rate=48000)
    assert abs(v.item() - r.item()) <= 1e-4 * abs(r.item())


def test_power_mel_rejects_unsupported(gpu):
    from mel_spectrogram import MelSpectrogram
    from sel import _lib as L
    with pytest.raises(NotImplementedError):
        MelSpectrogram(48000, norm="slaney")
    m = MelSpectrogram(48000, n_fft=14 * 2).to(gpu)  # 14 = 2*7: prime factor 7
    with pytest.raises(L.SelError):
        m(torch.randn(1, 4800, device=gpu))
