"""AudioDec generator without projector/quantizer ("without_PQC") — drop-in for
models/autoencoder_without_PQC/AudioDec.py (Generator :25-100).  The projector,
quantizer and decoder.conv1 are still constructed (same parameters / state_dict
as the reference) but forward is encoder -> decoder blocks -> conv2 (:94-100,
modules/decoder.py:116-123)."""
import torch

from models.autoencoder.AudioDec import Generator as _PQCGenerator
from models.autoencoder.AudioDec import StreamGenerator as _PQCStream
from models.autoencoder_without_PQC.modules.decoder import Decoder


class Generator(_PQCGenerator):
    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.decoder.__class__ = Decoder  # same parameters, conv1 skipped in forward

    def forward(self, x):
        h = self.encoder(self._flatten_channels(x))
        return self.decoder(h).float()


class StreamGenerator(Generator):
    """Streaming without_PQC generator (autoencoder_without_PQC/AudioDec.py:104-190):
    encode is the encoder alone, decode skips decoder.conv1 and takes (B, C, L)."""

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        if self.mode != "causal":
            raise NotImplementedError(f"AudioDec Streamer is not supported in {self.mode} mode (causal only)")
        self.reset_buffer()

    @torch.no_grad()
    def initial_encoder(self, receptive_length, device):
        self.quantizer.initial()
        return self.encode(torch.zeros(1, self.input_channels, receptive_length).to(device))

    @torch.no_grad()
    def initial_decoder(self, zq):
        self.decode(zq)

    @torch.no_grad()
    def encode(self, x):
        return self.encoder.encode(self._flatten_channels(x))

    @torch.no_grad()
    def quantize(self, z):
        zq, idx = self.quantizer.encode(z)
        return idx

    @torch.no_grad()
    def lookup(self, idx):
        return self.quantizer.decode(idx)

    @torch.no_grad()
    def decode(self, zq):
        return self.decoder.decode(zq)

    reset_buffer = _PQCStream.reset_buffer
