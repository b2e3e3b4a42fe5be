"""CPU checks of the drop-in boundary: libsel.so loads, exports exactly what
include/sel.h declares, the ctypes table covers it, and the product path refuses
CPU tensors instead of silently falling back."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

from conftest import REPO, golden

HEADER = os.path.join(REPO, "include", "sel.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(sel_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    from sel import _lib
    lib = _lib.load()
    names = declared_functions()
    assert len(names) >= 10
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    # the ctypes signature table is exactly the header
    assert sorted(_lib.SIGNATURES) == names


def test_library_reports_errors_without_gpu():
    from sel import _lib
    lib = _lib.load()
    # argument validation happens before any device work
    rc = lib.sel_stft_mag_fwd(None, 1, 100, 1000, 10, 100, None, 1e-7, None, None)
    assert rc < 0
    assert lib.sel_last_error()
    assert lib.sel_version() >= 1


def test_tune_keys_cover_every_knob():
    """Every knob the kernels read (keys up to 69 in round 6) is settable and
    reads back; a key out of range is refused and changes nothing (keys >= 64
    were silently ignored before round 6, so A/B runs on them compared a
    setting with itself)."""
    from sel import _lib
    lib = _lib.load()
    for key in (0, 63, 64, 67, 127):
        prev = lib.sel_tune(key, 7)
        assert prev >= 0 and lib.sel_tune_get(key) == 7, key
        assert lib.sel_tune(key, prev) == 7
    assert lib.sel_tune(128, 1) == -1 and lib.sel_tune_get(128) == -1


def test_product_refuses_cpu_tensors():
    from losses import MultiMelSpectrogramLoss, MultiResolutionSTFTLoss
    x = torch.randn(2, 1, 4800)
    with pytest.raises(RuntimeError):
        MultiMelSpectrogramLoss()(x, x)
    with pytest.raises(RuntimeError):
        MultiResolutionSTFTLoss()(x, x)


def test_product_melbank_matches_reference_buffers():
    from sel.melbank import slaney_mel
    g = golden("melmat")
    cfgs = {"24k_fmax24000": (24000, 2048, 80, 0, 24000), "24k_fmax12000": (24000, 2048, 80, 0, 12000),
            "48k_fmax24000": (48000, 2048, 80, 0, 24000), "default": (22050, 1024, 80, 80, 7600)}
    for k, (sr, n, m, lo, hi) in cfgs.items():
        np.testing.assert_array_equal(slaney_mel(sr, n, m, lo, hi).T, g[f"melmat.{k}"])


def test_mel_ranges_cover_nonzeros():
    from sel.melbank import slaney_mel
    from sel.spectral import mel_ranges
    mm = slaney_mel(24000, 2048, 80, 0, 24000).T
    kr, mr = mel_ranges(torch.from_numpy(mm))
    kr, mr = kr.numpy(), mr.numpy()
    for m in range(80):
        nz = np.nonzero(mm[:, m])[0]
        if nz.size:
            assert kr[m, 0] <= nz.min() and kr[m, 1] > nz.max()
        else:
            assert kr[m, 0] == kr[m, 1]
    for k in range(mm.shape[0]):
        nz = np.nonzero(mm[k])[0]
        if nz.size:
            assert mr[k, 0] <= nz.min() and mr[k, 1] > nz.max()


def test_product_htk_filterbank_matches_oracle():
    """The product's torchaudio-HTK filterbank restatement equals the oracle's."""
    from oracle import ref_ops as R
    from sel.melbank import htk_fbanks
    for args in [(201, 0.0, 24000.0, 128, 48000), (121, 0.0, 12000.0, 40, 24000), (257, 20.0, 8000.0, 80, 16000)]:
        assert torch.equal(htk_fbanks(*args), R.htk_melscale_fbanks(*args))
