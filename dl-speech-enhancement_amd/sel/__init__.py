"""sel — MI355X-native kernels for the denoise-training hot path of
s194584/dl-speech-enhancement (libsel.so via ctypes + autograd plumbing)."""
from ._lib import SelError, load, lib  # noqa: F401
