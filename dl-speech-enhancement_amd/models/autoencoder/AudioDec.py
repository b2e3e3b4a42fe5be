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
        # the quantizer works in fp32 (ResidualVQFn): the projector's conv writes
        # z as fp32 from its epilogue instead of bf16 + a cast launch each way
        conv = self.projector.project
        conv = conv[0] if isinstance(conv, torch.nn.Sequential) else conv   # 'conv1d_bn': the BN reads fp32
        if hasattr(conv, "out_float"):
            conv.out_float = True

    def _flatten_channels(self, x):
        B, C, T = x.size()
        return x.reshape(-1, self.input_channels, T) if C != self.input_channels else x

    def forward(self, x):
        h = self.encoder(self._flatten_channels(x))
        z = self.projector(h)
        zq, vqloss, perplexity = self.quantizer(z)
        y = self.decoder(zq)
        return y.float(), zq, z, vqloss, perplexity


# STREAMING
class StreamGenerator(Generator):
    """AudioDec streaming generator (AudioDec.py:106-191): the causal layers'
    pad_buffer carries the left context between calls; every step runs the same
    HIP conv kernels as training (layers.conv_layer *.inference)."""

    def __init__(self, input_channels=1, output_channels=1, encode_channels=32, decode_channels=32,
                 code_dim=64, codebook_num=8, codebook_size=1024, bias=True, enc_ratios=(2, 4, 8, 16),
                 dec_ratios=(16, 8, 4, 2), enc_strides=(3, 4, 5, 5), dec_strides=(5, 5, 4, 3),
                 mode="causal", codec="audiodec", projector="conv1d", quantier="residual_vq"):
        super().__init__(input_channels=input_channels, output_channels=output_channels,
                         encode_channels=encode_channels, decode_channels=decode_channels, code_dim=code_dim,
                         codebook_num=codebook_num, codebook_size=codebook_size, bias=bias,
                         enc_ratios=enc_ratios, dec_ratios=dec_ratios, enc_strides=enc_strides,
                         dec_strides=dec_strides, mode=mode, codec=codec, projector=projector,
                         quantier=quantier)
        if mode != "causal":
            raise NotImplementedError(f"AudioDec Streamer is not supported in {mode} mode (causal only)")
        self.reset_buffer()

    @torch.no_grad()
    def initial_encoder(self, receptive_length, device):
        self.quantizer.initial()
        z = self.encode(torch.zeros(1, self.input_channels, receptive_length).to(device))
        idx = self.quantize(z)
        return self.lookup(idx)

    @torch.no_grad()
    def initial_decoder(self, zq):
        self.decode(zq)

    @torch.no_grad()
    def encode(self, x):
        x = self._flatten_channels(x)
        return self.projector.encode(self.encoder.encode(x))

    @torch.no_grad()
    def quantize(self, z):
        zq, idx = self.quantizer.encode(z)
        return idx

    @torch.no_grad()
    def lookup(self, idx):
        return self.quantizer.decode(idx)

    @torch.no_grad()
    def decode(self, zq):
        return self.decoder.decode(zq.transpose(2, 1))

    def reset_buffer(self):
        """Zero every causal layer's pad_buffer (AudioDec.py:185-191)."""
        from layers.conv_layer import CausalConv1d, CausalConvTranspose1d

        def _reset(m):
            if isinstance(m, (CausalConv1d, CausalConvTranspose1d)):
                m.reset_buffer()
        self.apply(_reset)
