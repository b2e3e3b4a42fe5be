"""dataloader/data_utils.py drop-in: add_noise (:12-22) on device, dataloaders (:25-51)."""
import math
import random

import numpy as np
import torch
from torch.utils.data import DataLoader, random_split

from dataloader.collater import CollaterAudio, DeviceCollaterAudio
from sel import _lib as L


def add_noise(speech, noise, snr):
    """(scale * speech + noise) / 2 with scale = exp(snr/10) * ||noise|| / ||speech||
    over the WHOLE batch (reference :12-22).  Runs the sel_add_noise HIP kernel;
    device tensors only (the MI355X path has no CPU fallback)."""
    assert speech.shape == noise.shape, "Shapes are not equal!"
    L.need_device(speech, noise)
    snr = float(snr.item() if torch.is_tensor(snr) else snr)
    a = speech.contiguous().float()
    b = noise.contiguous().float()
    out = torch.empty_like(a)
    ws = L.workspace(L.lib().sel_add_noise_workspace(a.numel()), a.device)
    L.call("sel_add_noise", L.ptr(a), L.ptr(b), a.numel(), snr, L.ptr(out), L.ptr(ws), ws.numel(), L.stream())
    return out


def seed_worker(worker_id):
    worker_seed = torch.initial_seed() % 2 ** 32
    np.random.seed(worker_seed)
    random.seed(worker_seed)


def _device_mode(dataset):
    while hasattr(dataset, "dataset"):  # random_split Subset -> the AudioDataset
        dataset = dataset.dataset
    return getattr(dataset, "resample_device", False), getattr(dataset, "sample_rate", None)


def create_dataloader(dataset, batch_size, batch_length, generator, sampler=None):
    on_device, rate = _device_mode(dataset)
    if on_device:  # GPU resampling + crops in the main process (no workers: the collater uses the GPU)
        return DataLoader(dataset, batch_size=batch_size, shuffle=sampler is None, sampler=sampler,
                          generator=generator if sampler is None else None,
                          collate_fn=DeviceCollaterAudio(batch_length, rate), drop_last=True)
    return DataLoader(dataset, batch_size=batch_size, shuffle=sampler is None, sampler=sampler,
                      generator=generator if sampler is None else None, collate_fn=CollaterAudio(batch_length),
                      worker_init_fn=seed_worker, drop_last=True, pin_memory=torch.cuda.is_available())


def get_dataloaders(dataset, splits=None, batch_size=8, batch_length=2 * 48000, seed=82, rank=0, world_size=1):
    """70/15/15 split (reference :38-51).  With world_size > 1 every rank draws a
    disjoint, equally sized shard of each split (DistributedSampler semantics) so
    the global batch is world_size * batch_size."""
    if splits is None:
        splits = [0.7, 0.15, 0.15]
    generator = torch.manual_seed(seed)
    parts = random_split(dataset, splits, generator)
    out = []
    for frag in parts:
        sampler = None
        if world_size > 1:
            sampler = torch.utils.data.DistributedSampler(frag, num_replicas=world_size, rank=rank,
                                                          shuffle=True, seed=seed, drop_last=True)
        out.append(create_dataloader(frag, batch_size, batch_length, generator, sampler))
    return out


def set_epoch(loaders, epoch):
    """Reshuffle the data-parallel shards for a new epoch (DistributedSampler
    .set_epoch).  Single-process loaders reshuffle on their own: their shuffling
    generator advances every epoch, as in the reference; without this call a
    DistributedSampler would replay epoch 0's order forever."""
    for dl in loaders:
        sampler = getattr(dl, "sampler", None)
        if hasattr(sampler, "set_epoch"):
            sampler.set_epoch(epoch)


_ = math  # math.exp semantics documented above
