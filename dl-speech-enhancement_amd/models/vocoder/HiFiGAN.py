"""HiFi-GAN discriminator — drop-in for the reference ``models/vocoder/HiFiGAN.py``
``Discriminator`` (:308-395): MSD + MPD, outputs concatenated (MSD first).

The HiFi-GAN *generator* of the same reference file (:28-305) is the vocoder
of the codec's pre-training and is outside the denoise hot path (SURVEY §2 row
13); only the discriminator GAN mode needs (BASELINE config C5) is built.
"""
import torch
import torch.nn as nn

from models.vocoder.modules.discriminator import HiFiGANMultiPeriodDiscriminator, HiFiGANMultiScaleDiscriminator
from sel.streams import run_concurrent


class Discriminator(nn.Module):
    """HiFi-GAN multi-scale + multi-period discriminator module."""

    def __init__(self, scales=3, scale_downsample_pooling="AvgPool1d",
                 scale_downsample_pooling_params={"kernel_size": 4, "stride": 2, "padding": 2},
                 scale_discriminator_params={"in_channels": 1, "out_channels": 1, "kernel_sizes": [15, 41, 5, 3],
                                             "channels": 128, "max_downsample_channels": 1024, "max_groups": 16,
                                             "bias": True, "downsample_scales": [2, 2, 4, 4, 1],
                                             "nonlinear_activation": "LeakyReLU",
                                             "nonlinear_activation_params": {"negative_slope": 0.1}},
                 follow_official_norm=True, periods=[2, 3, 5, 7, 11],
                 period_discriminator_params={"in_channels": 1, "out_channels": 1, "kernel_sizes": [5, 3],
                                              "channels": 32, "downsample_scales": [3, 3, 3, 3, 1],
                                              "max_downsample_channels": 1024, "bias": True,
                                              "nonlinear_activation": "LeakyReLU",
                                              "nonlinear_activation_params": {"negative_slope": 0.1},
                                              "use_weight_norm": True, "use_spectral_norm": False}):
        super().__init__()
        self.msd = HiFiGANMultiScaleDiscriminator(scales=scales, downsample_pooling=scale_downsample_pooling,
                                                  downsample_pooling_params=scale_downsample_pooling_params,
                                                  discriminator_params=scale_discriminator_params,
                                                  follow_official_norm=follow_official_norm)
        self.mpd = HiFiGANMultiPeriodDiscriminator(periods=periods, discriminator_params=period_discriminator_params)

    def _chains(self, x, pooled, method):
        """The 3 scale and 5 period sub-discriminators on `method` (None = the
        module call), as independent chains on side streams (sel.streams: same
        kernels, same bits); MSD outputs first, as the reference concatenates."""
        fs = list(self.msd.discriminators) + list(self.mpd.discriminators)
        xs = list(pooled) + [x] * len(self.mpd.discriminators)
        calls = [(lambda f=f, v=v: f(v) if method is None else getattr(f, method)(v)) for f, v in zip(fs, xs)]
        return run_concurrent(calls, [x] + list(pooled))

    def _flat(self, x):
        batch, channel, time = x.size()
        return x.reshape(batch * channel, 1, time) if channel != 1 else x

    def forward(self, x):
        """x (B, C, T) -> list of lists of each sub-discriminator's layer outputs
        (MSD then MPD), HiFiGAN.py:380-395."""
        x = self._flat(x)
        return self._chains(x, self.msd._scales(x, lambda f, v: v), None)

    @torch.no_grad()
    def stash_first_half(self, x):
        """No-grad forward of B clips x into per-layer buffers sized for 2B clips,
        kept for forward_second_half (train_denoise.DenoiseStep: the generator
        step's D(target) is the D step's real half); returns x's outputs."""
        x = self._flat(x)
        return self._chains(x, self.msd._scales(x, lambda f, v: v), "stash_first_half")

    def clear_stash(self):
        """Drop every sub-discriminator's stash_first_half buffers (sized for 2B
        clips): called whenever the generator step will not be followed by a
        forward_second_half that consumes them."""
        for f in list(self.msd.discriminators) + list(self.mpd.discriminators):
            f._stash = None

    def forward_second_half(self, x):
        """forward(torch.cat([stashed clips, x])) without recomputing the stashed
        half, as one autograd graph over all 2B clips.  Each output row runs the
        same kernels as in the concatenated pass, but the flat tiling may put a
        clip in another tile: tests/test_gpu_gan.py holds the two paths to 1e-6
        (fp32) / 1e-3 (bf16) norm-wise, not to bit equality."""
        x = self._flat(x)
        with torch.no_grad():  # the waveform (a detached prediction) takes no gradient
            pooled = self.msd._scales(x, lambda f, v: v)
        return self._chains(x, pooled, "forward_second_half")
