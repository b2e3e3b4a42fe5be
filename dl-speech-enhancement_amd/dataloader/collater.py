"""Collaters — drop-in for dataloader/collater.py (host-side batching, :18-87)."""
import numpy as np
import torch


class CollaterAudio(object):
    """Random fixed-length crops -> (B, C, T) float32 (reference :18-60)."""

    def __init__(self, batch_length=9600):
        self.batch_length = batch_length

    def __call__(self, batch):
        xs = [b for b in batch if len(b) > self.batch_length]  # reference :35 (strictly longer)
        starts, ends = self._random_segment(xs)
        return self._cut(xs, starts, ends)

    def _random_segment(self, xs):
        starts = np.array([np.random.randint(0, len(x) - self.batch_length) for x in xs])
        return starts, starts + self.batch_length

    def _cut(self, xs, starts, ends):
        x_batch = np.array([x[s:e] for x, s, e in zip(xs, starts, ends)])
        return torch.tensor(x_batch, dtype=torch.float).transpose(2, 1)


class CollaterAudioPair(CollaterAudio):
    """(noisy, clean) pairs cut at the same offsets (reference :63-87)."""

    def __call__(self, batch):
        batch = [b for b in batch if len(b[0]) > self.batch_length and len(b[0]) == len(b[1])]
        assert len(batch) > 0, "No qualified audio pairs.!"
        xs, ns = [b[0] for b in batch], [b[1] for b in batch]
        starts, ends = self._random_segment(xs)
        return self._cut(ns, starts, ends), self._cut(xs, starts, ends)
