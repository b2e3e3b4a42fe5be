"""AudioDataset — drop-in for dataloader/AudioDataset.py (:7-36).

The reference loads with torchaudio (absent here) and resamples with
torchaudio.functional.resample (sinc_interp_hann).  Two modes:
  * resample="device" (SURVEY §8 f3): items are the raw files at their own rate;
    DeviceCollaterAudio[Pair] (dataloader/collater.py) resamples each whole file
    on the GPU with the torchaudio algorithm (sel.resample, HIP) and then cuts
    the reference's random crops — the reference's order of operations;
  * resample="host" (default): scipy PCM/float WAV read + polyphase
    scipy.signal.resample_poly on the host: same shapes ((T, 1) float32 per
    file), a different interpolation kernel."""
import glob
import os
from math import gcd

import numpy as np
from torch.utils.data import Dataset


def read_wav(path):
    """(T, C) float32 in [-1, 1) and the file's sample rate."""
    from scipy.io import wavfile
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        sr, d = wavfile.read(path)
    if d.dtype.kind == "i":
        d = d.astype(np.float32) / float(np.iinfo(d.dtype).max + 1)
    d = d.astype(np.float32)
    if d.ndim == 1:
        d = d[:, None]
    return d, int(sr)


def load_wav(path, sample_rate):
    from scipy.signal import resample_poly
    d, sr = read_wav(path)
    if sr != sample_rate:
        g = gcd(int(sr), int(sample_rate))
        d = resample_poly(d, sample_rate // g, sr // g, axis=0).astype(np.float32)
    return d


class AudioDataset(Dataset):
    def __init__(self, audio_dir, audio_root, sample_rate, resample="host"):
        if resample not in ("host", "device"):
            raise ValueError("resample must be 'host' or 'device'")
        self.audio_dir = audio_dir
        self.sample_rate = sample_rate
        self.resample_device = resample == "device"
        self.audio_file_names = []
        for depth in range(1, 3):
            files = glob.glob(audio_dir + "/*" * depth + ".wav")
            self.audio_file_names.extend(f.replace("\\", "/").split(audio_root + "/")[-1] for f in files)

    def __len__(self):
        return len(self.audio_file_names)

    def __getitem__(self, idx):
        path = os.path.join(self.audio_dir, self.audio_file_names[idx])
        if self.resample_device:
            return read_wav(path)  # (raw (T, C), sr): resampled on the GPU by the collater
        return load_wav(path, self.sample_rate)
