"""Waveform-based losses — drop-in for losses/waveform_loss.py (:15-74) on the
sel_shape_loss HIP kernels: L1 between max-pooled |y_hat| and |y| per window
length (MaxPool1d(w): stride w, floor), averaged over the lengths.  Gradients
flow to y_hat (the reference's usage: y is the ground truth); a y that requires
grad raises instead of being silently skipped."""
import ctypes

import torch

from sel import _lib as L


class _ShapeLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y_hat, y, win):
        L.need_device(y_hat, y)
        if y.requires_grad:
            raise L.SelError("sel: WaveformShapeLoss differentiates y_hat only (y is the ground truth)")
        yh = y_hat.float().contiguous()
        yt = y.float().contiguous()
        assert yh.shape == yt.shape, (yh.shape, yt.shape)
        T = yh.shape[-1]
        rows = yh.numel() // T
        nwin = T // win
        lib = L.lib()
        arg = torch.empty(rows * nwin, dtype=torch.int32, device=yh.device)
        sgn = torch.empty(rows * nwin, dtype=torch.float32, device=yh.device)
        out = torch.empty(1, dtype=torch.float32, device=yh.device)
        ws = L.workspace(lib.sel_shape_loss_workspace(rows, T, win), yh.device)
        L.call("sel_shape_loss_fwd", L.ptr(yh), L.ptr(yt), rows, T, win, L.ptr(arg), L.ptr(sgn), L.ptr(out),
               L.ptr(ws), ws.numel(), L.stream())
        ctx.save_for_backward(yh, arg, sgn)
        ctx.cfg = (rows, T, win, y_hat.dtype)
        return out[0]

    @staticmethod
    def backward(ctx, g):
        yh, arg, sgn = ctx.saved_tensors
        rows, T, win, dt = ctx.cfg
        gx = torch.zeros_like(yh)
        L.call("sel_shape_loss_bwd", L.ptr(yh), rows, T, win, L.ptr(arg), L.ptr(sgn),
               L.ptr(g.float().contiguous().view(1)), ctypes.c_float(1.0), L.ptr(gx), L.stream())
        return gx.to(dt), None, None


class WaveformShapeLoss(torch.nn.Module):
    """Waveform shape loss (waveform_loss.py:15-38)."""

    def __init__(self, winlen):
        super().__init__()
        self.loss = torch.nn.L1Loss()  # kept for attribute parity; the kernel computes it
        self.winlen = winlen
        self.maxpool = torch.nn.MaxPool1d(self.winlen)

    def forward(self, y_hat, y):
        return _ShapeLossFn.apply(y_hat, y, int(self.winlen))


class MultiWindowShapeLoss(torch.nn.Module):
    """Multi-window-length waveform shape loss (waveform_loss.py:41-74)."""

    def __init__(self, winlen=[300, 200, 100]):
        super().__init__()
        self.shape_losses = torch.nn.ModuleList()
        for wl in winlen:
            self.shape_losses += [WaveformShapeLoss(wl)]

    def forward(self, y_hat, y):
        loss = 0.0
        for f in self.shape_losses:
            loss += f(y_hat, y)
        loss /= len(self.shape_losses)
        return loss
