from .collater import *  # NOQA
from .data_utils import *  # NOQA
from .AudioDataset import *  # NOQA
