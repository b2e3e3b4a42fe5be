"""AudioDec generator (with projector + residual VQ) — drop-in for
models/autoencoder/AudioDec.py (Generator :26-103).  forward returns
(y, zq, z, vqloss, perplexity) exactly like the reference (:95-103)."""
import torch

from models.autoencoder.modules.decoder import Decoder
from models.autoencoder.modules.encoder import Encoder
from models.autoencoder.modules.projector import Projector
from models.autoencoder.modules.quantizer import Quantizer


class Generator(torch.nn.Module):
    """AudioDec generator."""

    def __init__(self, input_channels=1, output_channels=1, encode_channels=32, decode_channels=32,
                 code_dim=64, codebook_num=8, codebook_size=1024, bias=True, enc_ratios=(2, 4, 8, 16),
                 dec_ratios=(16, 8, 4, 2), enc_strides=(3, 4, 5, 5), dec_strides=(5, 5, 4, 3),
                 mode="causal", codec="audiodec", projector="conv1d", quantier="residual_vq"):
        super().__init__()
        if codec != "audiodec":
            raise NotImplementedError(f"Codec ({codec}) is not supported!")
        self.mode = mode
        self.input_channels = input_channels
        self.encoder = Encoder(input_channels=input_channels, encode_channels=encode_channels,
                               channel_ratios=enc_ratios, strides=enc_strides, kernel_size=7, bias=bias,
                               mode=mode)
        self.decoder = Decoder(code_dim=code_dim, output_channels=output_channels,
                               decode_channels=decode_channels, channel_ratios=dec_ratios,
                               strides=dec_strides, kernel_size=7, bias=bias, mode=mode)
        self.projector = Projector(input_channels=self.encoder.out_channels, code_dim=code_dim, kernel_size=3,
                                   stride=1, bias=False, mode=mode, model=projector)
        self.quantizer = Quantizer(code_dim=code_dim, codebook_num=codebook_num, codebook_size=codebook_size,
                                   model=quantier)

    def _flatten_channels(self, x):
        B, C, T = x.size()
        return x.reshape(-1, self.input_channels, T) if C != self.input_channels else x

    def forward(self, x):
        h = self.encoder(self._flatten_channels(x))
        z = self.projector(h)
        zq, vqloss, perplexity = self.quantizer(z)
        y = self.decoder(zq)
        return y.float(), zq, z, vqloss, perplexity
