"""AudioDataset — drop-in for dataloader/AudioDataset.py (:7-36).

The reference loads with torchaudio (absent here) and resamples with
torchaudio.functional.resample; this host-side loader reads PCM/float WAV with
scipy and resamples with a polyphase filter (scipy.signal.resample_poly): same
shapes ((T, 1) float32 per file), different interpolation kernel."""
import glob
import os
from math import gcd

import numpy as np
from torch.utils.data import Dataset


def load_wav(path, sample_rate):
    from scipy.io import wavfile
    from scipy.signal import resample_poly
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        sr, d = wavfile.read(path)
    if d.dtype.kind == "i":
        d = d.astype(np.float32) / float(np.iinfo(d.dtype).max + 1)
    d = d.astype(np.float32)
    if d.ndim == 1:
        d = d[:, None]
    if sr != sample_rate:
        g = gcd(int(sr), int(sample_rate))
        d = resample_poly(d, sample_rate // g, sr // g, axis=0).astype(np.float32)
    return d


class AudioDataset(Dataset):
    def __init__(self, audio_dir, audio_root, sample_rate):
        self.audio_dir = audio_dir
        self.sample_rate = sample_rate
        self.audio_file_names = []
        for depth in range(1, 3):
            files = glob.glob(audio_dir + "/*" * depth + ".wav")
            self.audio_file_names.extend(f.replace("\\", "/").split(audio_root + "/")[-1] for f in files)

    def __len__(self):
        return len(self.audio_file_names)

    def __getitem__(self, idx):
        return load_wav(os.path.join(self.audio_dir, self.audio_file_names[idx]), self.sample_rate)
