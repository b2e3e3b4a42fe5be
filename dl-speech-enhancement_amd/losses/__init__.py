from .mel_loss import *  # NOQA
from .stft_loss import *  # NOQA
from .waveform_loss import *  # NOQA
from .adversarial_loss import *  # NOQA
from .feat_match_loss import *  # NOQA
