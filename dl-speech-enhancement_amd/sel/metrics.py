"""SNR metric used as a loss term by train_denoise.py (:120, :140).

The reference uses torchmetrics 1.2.0 ``SignalNoiseRatio()`` (third-party,
absent here; parity unpinned beyond its published formula):
    snr_b = 10 * log10((sum_t target^2 + eps) / (sum_t (target - preds)^2 + eps)),
    eps = finfo(float32).eps, zero_mean=False, mean over the batch.
Computed by the sel_snr_fwd / sel_snr_bwd HIP kernels.
"""
import torch

from . import _lib as L


class _SNRFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pred, target):
        L.need_device(pred, target)
        T = pred.shape[-1]
        p = pred.contiguous().float().reshape(-1, T)
        t = target.contiguous().float().reshape(-1, T)
        B = p.shape[0]
        sums = torch.empty(2 * B, dtype=torch.float64, device=p.device)
        out = torch.empty((), dtype=torch.float32, device=p.device)
        L.call("sel_snr_fwd", L.ptr(p), L.ptr(t), B, T, L.ptr(sums), L.ptr(out), L.stream())
        ctx.save_for_backward(p, t, sums)
        ctx.shape = pred.shape
        return out

    @staticmethod
    def backward(ctx, g):
        p, t, sums = ctx.saved_tensors
        B, T = p.shape
        gp = torch.empty_like(p)
        L.call("sel_snr_bwd", L.ptr(p), L.ptr(t), B, T, L.ptr(sums), L.ptr(g.contiguous()), L.ptr(gp), L.stream())
        return gp.view(ctx.shape), None


class SignalNoiseRatio(torch.nn.Module):
    """Drop-in for torchmetrics.audio.SignalNoiseRatio as called by train_denoise.py."""

    def __init__(self, zero_mean=False):
        super().__init__()
        if zero_mean:
            raise NotImplementedError("sel: only zero_mean=False (the train_denoise.py default)")

    def forward(self, preds, target):
        return _SNRFn.apply(preds, target)
