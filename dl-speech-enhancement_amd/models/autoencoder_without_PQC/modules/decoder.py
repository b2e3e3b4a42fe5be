"""without_PQC decoder: the reference comments out ``x = self.conv1(z)``
(models/autoencoder_without_PQC/modules/decoder.py:116-123)."""
from models.autoencoder.modules.decoder import Decoder as _Decoder
from models.autoencoder.modules.decoder import DecoderBlock  # noqa: F401


class Decoder(_Decoder):
    skip_conv1 = True
