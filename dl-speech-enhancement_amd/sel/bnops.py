"""BatchNorm1d on the HIP kernels (glue.hip sel_batchnorm_fwd / _bwd): the
projector's 'conv1d_bn' form (models/autoencoder/modules/projector.py:40-44).

Same module, state_dict and semantics as torch.nn.BatchNorm1d (the reference
uses it directly): batch statistics with the biased variance in training,
running_mean / running_var updated with `momentum` and the unbiased variance,
num_batches_tracked counted; the running statistics in evaluation.  Inputs
are (B, C, T) views of channels-last (B, T, C) storage, as every sel conv
output; computed in fp32 (a bf16 input is cast first)."""
import ctypes

import torch
import torch.nn as nn

from . import _lib as L
from . import convops as CO


class BatchNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, running_mean, running_var, training, eps, momentum):
        # x: (rows, C) fp32 contiguous
        L.need_device(x)
        rows, C = x.shape
        lib = L.lib()
        ws = L.workspace(lib.sel_batchnorm_workspace(rows, C), x.device)
        mean = torch.empty(C, dtype=torch.float32, device=x.device)
        invstd = torch.empty_like(mean)
        y = torch.empty_like(x)
        g = gamma.detach().contiguous() if gamma is not None else None
        b = beta.detach().contiguous() if beta is not None else None
        L.call("sel_batchnorm_fwd", L.ptr(x), rows, C, L.ptr(g), L.ptr(b), int(training), float(eps),
               float(momentum), L.ptr(running_mean), L.ptr(running_var), L.ptr(mean), L.ptr(invstd), L.ptr(y),
               L.ptr(ws), ws.numel(), L.stream())
        ctx.save_for_backward(x, g, mean, invstd)
        ctx.training = training
        return y

    @staticmethod
    def backward(ctx, gy):
        x, g, mean, invstd = ctx.saved_tensors
        rows, C = x.shape
        gy = gy.contiguous().float()
        lib = L.lib()
        ws = L.workspace(lib.sel_batchnorm_workspace(rows, C), x.device)
        gx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        gg = torch.empty(C, dtype=torch.float32, device=x.device) if g is not None else None
        gb = torch.empty(C, dtype=torch.float32, device=x.device) if g is not None else None
        L.call("sel_batchnorm_bwd", L.ptr(x), L.ptr(gy), rows, C, L.ptr(g), L.ptr(mean), L.ptr(invstd),
               int(ctx.training), L.ptr(gx), L.ptr(gg), L.ptr(gb), L.ptr(ws), ws.numel(), L.stream())
        return gx, gg, gb, None, None, None, None, None


class BatchNorm1d(nn.BatchNorm1d):
    """torch.nn.BatchNorm1d (same constructor and state_dict) on the HIP kernels,
    for (B, C, T) inputs."""

    def forward(self, x):
        if x.dim() != 3:
            raise NotImplementedError("sel BatchNorm1d takes (B, C, T) inputs")
        B, C, T = x.shape
        xc = CO.cast(CO.to_cl(x), torch.float32)
        training = self.training or not self.track_running_stats
        momentum = 0.0 if self.momentum is None else self.momentum
        if self.training and self.track_running_stats:
            self.num_batches_tracked.add_(1)
            if self.momentum is None:   # cumulative moving average (torch's momentum=None)
                momentum = 1.0 / float(self.num_batches_tracked)
        upd = self.training and self.track_running_stats
        y = BatchNormFn.apply(xc.reshape(B * T, C), self.weight if self.affine else None,
                              self.bias if self.affine else None,
                              self.running_mean if (upd or not training) else None,
                              self.running_var if (upd or not training) else None,
                              training, self.eps, momentum)
        return y.view(B, T, C).transpose(1, 2)
