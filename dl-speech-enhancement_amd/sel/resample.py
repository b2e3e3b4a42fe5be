"""On-device band-limited resampling — torchaudio.functional.resample's
sinc_interp_hann path (the call at dataloader/AudioDataset.py:28-33) on the
sel_resample HIP kernel (csrc/resample.hip restates the algorithm)."""
import ctypes
import functools
import math

import torch

from sel import _lib as L


@functools.lru_cache(maxsize=64)
def _table_host(orig_freq, new_freq, lowpass_filter_width, rolloff):
    lib = L.load()
    nph, ntaps = ctypes.c_int(), ctypes.c_int()
    L.check(lib.sel_resample_plan(orig_freq, new_freq, lowpass_filter_width, rolloff, ctypes.byref(nph),
                                  ctypes.byref(ntaps)), "sel_resample_plan")
    t = torch.empty(nph.value, ntaps.value, dtype=torch.float32)
    L.check(lib.sel_resample_kernel(orig_freq, new_freq, lowpass_filter_width, rolloff,
                                    ctypes.c_void_p(t.data_ptr())), "sel_resample_kernel")
    return t


_DEV_TABLES = {}


def resample(waveform, orig_freq, new_freq, lowpass_filter_width=6, rolloff=0.99,
             resampling_method="sinc_interp_hann"):
    """Drop-in for torchaudio.functional.resample (sinc_interp_hann): (..., time)
    fp32 on the device -> (..., ceil(time * new / orig)) with the reduced ratio."""
    if resampling_method not in ("sinc_interp_hann", "sinc_interpolation"):
        raise NotImplementedError(f"sel.resample: {resampling_method} is not implemented")
    if orig_freq <= 0 or new_freq <= 0:
        raise ValueError("Original frequency and desired frequecy should be positive")
    if orig_freq == new_freq:
        return waveform
    L.need_device(waveform)
    lib = L.lib()
    g = math.gcd(int(orig_freq), int(new_freq))
    o, n = int(orig_freq) // g, int(new_freq) // g
    key = (o, n, int(lowpass_filter_width), float(rolloff), waveform.device)
    tab = _DEV_TABLES.get(key)
    if tab is None:
        tab = _table_host(o, n, int(lowpass_filter_width), float(rolloff)).to(waveform.device)
        _DEV_TABLES[key] = tab
    shape = waveform.shape
    x = waveform.reshape(-1, shape[-1]).float().contiguous()
    out_len = lib.sel_resample_out_len(x.shape[1], o, n)
    y = torch.empty(x.shape[0], out_len, dtype=torch.float32, device=x.device)
    L.call("sel_resample", L.ptr(x), x.shape[0], x.shape[1], o, n, int(lowpass_filter_width), float(rolloff),
           L.ptr(tab), L.ptr(y), L.stream())
    return y.view(*shape[:-1], out_len)
