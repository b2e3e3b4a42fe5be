"""GPU parity of the device data pipeline: sel.resample (HIP)
against the oracle restatement of torchaudio 2.1.1's functional.resample
(oracle/ref_ops.resample, fp64) within 1e-5 relative; and the device
collater (resample each whole file, then the reference's random crops,
collater.py:33-60) against the same steps in the oracle."""
import math
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

RATIOS = [(48000, 24000), (16000, 24000), (44100, 24000), (24000, 48000), (22050, 24000), (24000, 24000)]


@pytest.mark.parametrize("orig,new", RATIOS)
@pytest.mark.parametrize("shape", [(3, 9601), (1, 2, 4000), (5,)])
def test_resample_vs_oracle(gpu, orig, new, shape):
    from oracle import ref_ops as R
    from sel.resample import resample
    g = torch.Generator().manual_seed(orig + new + shape[-1])
    x = 0.3 * torch.randn(*shape, generator=g)
    y = resample(x.to(gpu), orig, new)
    yr = R.resample(x.double(), orig, new)
    assert y.shape == yr.shape
    e = ((y.double().cpu() - yr).norm() / yr.norm()).item()
    assert e < 1e-5, e


def test_resample_errors(gpu):
    from sel.resample import resample
    with pytest.raises(RuntimeError, match="CPU"):
        resample(torch.randn(100), 48000, 24000)
    with pytest.raises(NotImplementedError):
        resample(torch.randn(100, device=gpu), 48000, 24000, resampling_method="sinc_interp_kaiser")


def test_device_collater_matches_oracle_pipeline(gpu, tmp_path):
    from scipy.io import wavfile
    from oracle import ref_ops as R
    from dataloader.AudioDataset import AudioDataset
    from dataloader.collater import DeviceCollaterAudio
    rng = np.random.default_rng(4)
    root = tmp_path / "audio"
    os.makedirs(root / "spk", exist_ok=True)
    for i, n in enumerate((48000, 60000, 52000)):
        pcm = (rng.standard_normal(n) * 3000).astype(np.int16)
        wavfile.write(str(root / "spk" / f"f{i}.wav"), 48000, pcm)
    ds = AudioDataset(str(root), str(root), 24000, resample="device")
    items = [ds[i] for i in range(len(ds))]
    col = DeviceCollaterAudio(batch_length=9600, sample_rate=24000, device=gpu)
    np.random.seed(7)
    xb = col(items)
    np.random.seed(7)
    ref = [R.resample(torch.from_numpy(x).double().transpose(0, 1), sr, 24000).transpose(0, 1) for x, sr in items]
    ref = [r for r in ref if len(r) > 9600]
    starts = [np.random.randint(0, len(r) - 9600) for r in ref]
    rb = torch.stack([r[s:s + 9600] for r, s in zip(ref, starts)]).transpose(2, 1)
    assert xb.shape == rb.shape == (3, 1, 9600) and xb.is_cuda
    e = ((xb.double().cpu() - rb).norm() / rb.norm()).item()
    assert e < 1e-5, e
