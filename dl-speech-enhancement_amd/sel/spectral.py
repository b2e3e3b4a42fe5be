"""Autograd ops over the spectral kernels of libsel.so.

Reference semantics restated here (file:line under the reference root):
* stft magnitude            losses/stft_loss.py:19-35
* SC / log-mag losses        losses/stft_loss.py:45-56, :66-77
* fused per-resolution loss  losses/stft_loss.py:100-117
* log-mel spectrogram        losses/mel_loss.py:74-94
* mel L1                     losses/mel_loss.py:151-154
"""
import numpy as np
import os

import torch

from . import _lib as L
from . import dist as D

LOG_KIND = {None: 0, 2.0: 1, 10.0: 2}


def _signal_2d(x):
    if x.dim() == 3:
        x = x.reshape(-1, x.size(2))
    if x.dim() != 2:
        raise ValueError(f"expected (B, T) or (B, C, T) waveform, got {tuple(x.shape)}")
    if x.dtype != torch.float32:
        raise TypeError(f"sel spectral ops compute in fp32 (got {x.dtype})")
    return x.contiguous()


def _frames(T, hop):
    return 1 + T // hop


def _fft_flops(n):
    """Radix-2 count of one real-input length-n FFT (2.5 n log2 n)."""
    import math
    return 2.5 * n * math.log2(n)


def _spec_meta(tag, B, T, hop, n_fft, n_io, n_fft_per_frame, extra_per_frame=0.0):
    """(tag, algorithmic bytes, flops) of a fused spectral launch for bench.py's
    timer: n_io fp32 (B, T) waveforms read or written once (frames are formed
    in-kernel; their overlap is served on chip), n_fft_per_frame transforms
    per frame."""
    F = _frames(T, hop)
    return (f"{tag}[n_fft={n_fft}]", 4 * n_io * B * T,
            B * F * (n_fft_per_frame * _fft_flops(n_fft) + extra_per_frame))


class StftMag(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, n_fft, hop, win_length, window, eps):
        L.need_device(x, window)
        lib = L.lib()
        B, T = x.shape
        F, K = _frames(T, hop), n_fft // 2 + 1
        mag = torch.empty(B, F, K, device=x.device, dtype=torch.float32)
        L.call("sel_stft_mag_fwd", L.ptr(x), B, T, n_fft, hop, win_length, L.ptr(window),
                                     float(eps), L.ptr(mag), L.stream())
        ctx.save_for_backward(x, window)
        ctx.cfg = (n_fft, hop, win_length, float(eps))
        return mag

    @staticmethod
    def backward(ctx, g):
        x, window = ctx.saved_tensors
        n_fft, hop, win, eps = ctx.cfg
        lib = L.lib()
        B, T = x.shape
        g = g.contiguous()
        gx = torch.empty_like(x)
        nb = lib.sel_stft_bwd_workspace(B, T, n_fft, hop, win)
        ws = L.workspace(nb, x.device)
        L.call("sel_stft_mag_bwd", L.ptr(x), B, T, n_fft, hop, win, L.ptr(window), eps, L.ptr(g),
                                     L.ptr(gx), L.ptr(ws), ws.numel(), L.stream())
        return gx, None, None, None, None, None


def stft_mag(x, n_fft, hop, win_length, window, eps=1e-7):
    return StftMag.apply(_signal_2d(x), int(n_fft), int(hop), int(win_length),
                         window.contiguous().float(), eps)


class MagPairLoss(torch.autograd.Function):
    """(x_mag, y_mag) -> [sc, logmag]  (stft_loss.py:56 and :77)."""

    @staticmethod
    def forward(ctx, x_mag, y_mag):
        L.need_device(x_mag, y_mag)
        lib = L.lib()
        xm, ym = x_mag.contiguous(), y_mag.contiguous()
        n = xm.numel()
        sums = torch.empty(3, dtype=torch.float64, device=xm.device)
        ws = L.workspace(lib.sel_mag_pair_workspace(n), xm.device)
        L.call("sel_mag_pair_sums", L.ptr(xm), L.ptr(ym), n, L.ptr(sums), L.ptr(ws), ws.numel(),
                                      L.stream())
        sums, n_all, ctx.scale = D.global_loss_sums(sums, n)  # data parallel: global-batch SC
        out = torch.empty(2, dtype=torch.float32, device=xm.device)
        L.call("sel_stft_loss_finish", L.ptr(sums), n_all, L.ptr(out), L.stream())
        ctx.save_for_backward(xm, ym, sums)
        ctx.n_all = n_all
        return out

    @staticmethod
    def backward(ctx, g):
        xm, ym, sums = ctx.saved_tensors
        lib = L.lib()
        g = (g * ctx.scale if ctx.scale != 1.0 else g).contiguous()
        coef = torch.empty(4, dtype=torch.float32, device=xm.device)
        L.call("sel_stft_loss_coef", L.ptr(sums), ctx.n_all, L.ptr(g[0:1]), L.ptr(g[1:2]),
                                       L.ptr(coef), L.stream())
        gx = torch.empty_like(xm)
        gy = torch.empty_like(ym) if ctx.needs_input_grad[1] else None
        L.call("sel_mag_pair_bwd", L.ptr(xm), L.ptr(ym), xm.numel(), L.ptr(coef), L.ptr(gx),
                                     L.ptr(gy), L.stream())
        return gx, gy


class StftLoss(torch.autograd.Function):
    """Fused one-resolution STFT loss: (x, y) -> [sc, logmag]; grad w.r.t. x only
    (y is the ground truth in every reference call site, trainerGAN.py:227)."""

    @staticmethod
    def forward(ctx, x, y, n_fft, hop, win_length, window):
        L.need_device(x, y, window)
        lib = L.lib()
        B, T = x.shape
        if y.shape != x.shape:
            raise ValueError(f"shape mismatch {tuple(x.shape)} vs {tuple(y.shape)}")
        sums = torch.empty(3, dtype=torch.float64, device=x.device)
        ws = L.workspace(lib.sel_stft_loss_workspace(B, T, n_fft, hop, win_length), x.device)
        L.call("sel_stft_loss_fwd", L.ptr(x), L.ptr(y), B, T, n_fft, hop, win_length, L.ptr(window),
               L.ptr(sums), L.ptr(ws), ws.numel(), L.stream(),
               meta=lambda: _spec_meta("k_stft_loss_fwd", B, T, hop, n_fft, 2, 2))
        n = B * _frames(T, hop) * (n_fft // 2 + 1)
        sums, n, ctx.scale = D.global_loss_sums(sums, n)  # data parallel: global-batch SC
        out = torch.empty(2, dtype=torch.float32, device=x.device)
        L.call("sel_stft_loss_finish", L.ptr(sums), n, L.ptr(out), L.stream())
        ctx.save_for_backward(x, y, window, sums)
        ctx.cfg = (n_fft, hop, win_length, n)
        return out

    @staticmethod
    def backward(ctx, g):
        x, y, window, sums = ctx.saved_tensors
        n_fft, hop, win, n = ctx.cfg
        lib = L.lib()
        B, T = x.shape
        g = (g * ctx.scale if ctx.scale != 1.0 else g).contiguous()
        coef = torch.empty(4, dtype=torch.float32, device=x.device)
        L.call("sel_stft_loss_coef", L.ptr(sums), n, L.ptr(g[0:1]), L.ptr(g[1:2]), L.ptr(coef),
                                       L.stream())
        gx = torch.empty_like(x)
        ws = L.workspace(lib.sel_stft_loss_workspace(B, T, n_fft, hop, win), x.device)
        L.call("sel_stft_loss_bwd", L.ptr(x), L.ptr(y), B, T, n_fft, hop, win, L.ptr(window),
               L.ptr(coef), L.ptr(gx), L.ptr(ws), ws.numel(), L.stream(),
               meta=lambda: _spec_meta("k_stft_loss_bwd", B, T, hop, n_fft, 3, 3))
        return gx, None, None, None, None, None


def stft_loss(x, y, n_fft, hop, win_length, window):
    out = StftLoss.apply(_signal_2d(x), _signal_2d(y).detach(), int(n_fft), int(hop),
                         int(win_length), window.contiguous().float())
    return out[0], out[1]


def mel_ranges(melmat):
    """Nonzero structure of a (K, M) filterbank -> (krange (M,2), mrange (K,2)) int32."""
    mm = np.asarray(melmat.detach().cpu().numpy() if torch.is_tensor(melmat) else melmat)
    K, M = mm.shape
    nz = mm != 0
    kr = np.zeros((M, 2), dtype=np.int32)
    for m in range(M):
        idx = np.nonzero(nz[:, m])[0]
        if idx.size:
            kr[m] = (idx[0], idx[-1] + 1)
    mr = np.zeros((K, 2), dtype=np.int32)
    for k in range(K):
        idx = np.nonzero(nz[k])[0]
        if idx.size:
            mr[k] = (idx[0], idx[-1] + 1)
    return torch.from_numpy(kr), torch.from_numpy(mr)


class LogMel(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, n_fft, hop, win_length, window, melmat, krange, mrange, eps, log_kind):
        L.need_device(x, window, melmat, krange, mrange)
        lib = L.lib()
        B, T = x.shape
        M = melmat.shape[1]
        out = torch.empty(B, M, _frames(T, hop), device=x.device, dtype=torch.float32)
        L.call("sel_logmel_fwd", L.ptr(x), B, T, n_fft, hop, win_length, L.ptr(window), L.ptr(melmat),
                                   L.ptr(krange), M, float(eps), log_kind, L.ptr(out), L.stream())
        ctx.save_for_backward(x, window, melmat, krange, mrange)
        ctx.cfg = (n_fft, hop, win_length, float(eps), log_kind)
        return out

    @staticmethod
    def backward(ctx, g):
        x, window, melmat, krange, mrange = ctx.saved_tensors
        n_fft, hop, win, eps, log_kind = ctx.cfg
        lib = L.lib()
        B, T = x.shape
        g = g.contiguous()
        gx = torch.empty_like(x)
        ws = L.workspace(lib.sel_logmel_bwd_workspace(B, T, n_fft, hop, win), x.device)
        L.call("sel_logmel_bwd", L.ptr(x), B, T, n_fft, hop, win, L.ptr(window), L.ptr(melmat),
                                   L.ptr(krange), L.ptr(mrange), melmat.shape[1], eps, log_kind,
                                   L.ptr(g), None, None, 0.0, L.ptr(gx), L.ptr(ws), ws.numel(),
                                   L.stream())
        return gx, None, None, None, None, None, None, None, None, None


# SEL_MEL_PAIR=0: the two log-mel forwards of the L1 loss as two launches
MEL_PAIR_ONE_LAUNCH = os.environ.get("SEL_MEL_PAIR", "1") != "0"
# SEL_MEL_FUSED=0: the loss as log-mel forwards + L1 + a log-mel backward
# instead of the fused forward-with-gradient launch (sel_mel_l1_fwd_grad)
MEL_FUSED = os.environ.get("SEL_MEL_FUSED", "1") != "0"


class MelL1(torch.autograd.Function):
    """mean |logmel(x) - logmel(y)| with grad w.r.t. x (mel_loss.py:151-154).

    When x needs a gradient the forward is the fused launch: it returns the
    loss and keeps d loss / d x for a unit upstream (one (B, T) fp32 tensor),
    and the backward scales it by the upstream gradient."""

    @staticmethod
    def forward(ctx, x, y, n_fft, hop, win_length, window, melmat, krange, mrange, eps, log_kind):
        L.need_device(x, y, window, melmat, krange, mrange)
        lib = L.lib()
        B, T = x.shape
        M = melmat.shape[1]
        F = _frames(T, hop)
        s = L.stream()
        ctx.fused = MEL_FUSED and ctx.needs_input_grad[0]
        if ctx.fused:
            loss = torch.empty((), device=x.device, dtype=torch.float32)
            gx1 = torch.empty_like(x)
            ws = L.workspace(lib.sel_mel_l1_workspace(B, T, n_fft, hop, win_length), x.device)
            L.call("sel_mel_l1_fwd_grad", L.ptr(x), L.ptr(y), B, T, n_fft, hop, win_length, L.ptr(window),
                   L.ptr(melmat), L.ptr(krange), L.ptr(mrange), M, float(eps), log_kind, L.ptr(loss), L.ptr(gx1),
                   L.ptr(ws), ws.numel(), s,
                   meta=lambda: _spec_meta("k_mel_l1", B, T, hop, n_fft, 3, 3, 3 * 2.0 * (n_fft // 2 + 1) * M))
            ctx.save_for_backward(gx1)
            return loss
        if MEL_PAIR_ONE_LAUNCH:
            # both signals' log-mels in ONE launch over the (2B, T) pair: one frame
            # grid of twice the frames instead of two launches with their tails
            ab = torch.empty(2 * B, M, F, device=x.device, dtype=torch.float32)
            xy = torch.cat((x, y))
            L.call("sel_logmel_fwd", L.ptr(xy), 2 * B, T, n_fft, hop, win_length, L.ptr(window),
                   L.ptr(melmat), L.ptr(krange), M, float(eps), log_kind, L.ptr(ab), s)
            a, b = ab[:B], ab[B:]
        else:
            a = torch.empty(B, M, F, device=x.device, dtype=torch.float32)
            b = torch.empty_like(a)
            for src, dst in ((x, a), (y, b)):
                L.call("sel_logmel_fwd", L.ptr(src), B, T, n_fft, hop, win_length, L.ptr(window),
                                           L.ptr(melmat), L.ptr(krange), M, float(eps), log_kind,
                                           L.ptr(dst), s)
        n = a.numel()
        loss = torch.empty((), device=x.device, dtype=torch.float32)
        ws = L.workspace(lib.sel_l1_workspace(n), x.device)
        L.call("sel_l1_mean", L.ptr(a), L.ptr(b), n, L.ptr(loss), L.ptr(ws), ws.numel(), s)
        ctx.save_for_backward(x, window, melmat, krange, mrange, a, b)
        ctx.cfg = (n_fft, hop, win_length, float(eps), log_kind)
        return loss

    @staticmethod
    def backward(ctx, g):
        if ctx.fused:
            (gx1,) = ctx.saved_tensors
            return gx1 * g, None, None, None, None, None, None, None, None, None, None
        x, window, melmat, krange, mrange, a, b = ctx.saved_tensors
        n_fft, hop, win, eps, log_kind = ctx.cfg
        lib = L.lib()
        B, T = x.shape
        g = g.contiguous()
        gx = torch.empty_like(x)
        ws = L.workspace(lib.sel_logmel_bwd_workspace(B, T, n_fft, hop, win), x.device)
        L.call("sel_logmel_bwd", L.ptr(x), B, T, n_fft, hop, win, L.ptr(window), L.ptr(melmat),
                                   L.ptr(krange), L.ptr(mrange), melmat.shape[1], eps, log_kind,
                                   L.ptr(a), L.ptr(b), L.ptr(g), 1.0 / a.numel(), L.ptr(gx), L.ptr(ws),
                                   ws.numel(), L.stream())
        return gx, None, None, None, None, None, None, None, None, None, None


def power_mel(x, n_fft, hop, win_length, window, fb, krange, power=2.0):
    """|STFT|^power @ fb (torchaudio MelSpectrogram semantics, mel_spectrogram.py:38).
    x (B, T) fp32 device -> (B, n_mels, 1 + T // hop).  Forward only: the reference
    uses it as an eval metric (Mel_L1), so a grad-requiring input is refused
    rather than silently detached."""
    if torch.is_grad_enabled() and x.requires_grad:
        raise NotImplementedError("sel power_mel is forward-only (eval metric); call under torch.no_grad()")
    x = _signal_2d(x)
    L.need_device(x, window, fb, krange)
    B, T = x.shape
    n_mels = fb.shape[1]
    out = torch.empty(B, n_mels, _frames(T, hop), device=x.device, dtype=torch.float32)
    L.call("sel_power_mel_fwd", L.ptr(x), B, T, int(n_fft), int(hop), int(win_length), L.ptr(window),
           L.ptr(fb), L.ptr(krange), n_mels, float(power), L.ptr(out), L.stream())
    return out
