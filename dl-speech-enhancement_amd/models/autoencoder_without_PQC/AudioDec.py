"""AudioDec generator without projector/quantizer ("without_PQC") — drop-in for
models/autoencoder_without_PQC/AudioDec.py (Generator :25-100).  The projector,
quantizer and decoder.conv1 are still constructed (same parameters / state_dict
as the reference) but forward is encoder -> decoder blocks -> conv2 (:94-100,
modules/decoder.py:116-123)."""
from models.autoencoder.AudioDec import Generator as _PQCGenerator
from models.autoencoder_without_PQC.modules.decoder import Decoder


class Generator(_PQCGenerator):
    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.decoder.__class__ = Decoder  # same parameters, conv1 skipped in forward

    def forward(self, x):
        h = self.encoder(self._flatten_channels(x))
        return self.decoder(h).float()
