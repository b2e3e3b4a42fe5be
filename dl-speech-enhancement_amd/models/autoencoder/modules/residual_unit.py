"""Residual units — drop-in for models/autoencoder/modules/residual_unit.py.

forward = x + conv2(ELU(conv1(ELU(x)))) (reference :43-46), executed as one
fused autograd op (sel.convops.ResidualUnitFn): ELU is applied while the conv
input tile is staged, the residual add in the 1x1 conv's epilogue.
"""
import torch
import torch.nn as nn

from layers.conv_layer import CausalConv1d, Conv1d1x1, NonCausalConv1d
from sel import convops as CO


class NonCausalResidualUnit(nn.Module):
    def __init__(self, in_channels, out_channels, kernel_size=7, dilation=1, bias=False,
                 nonlinear_activation="ELU", nonlinear_activation_params={}):
        super().__init__()
        if nonlinear_activation != "ELU" or nonlinear_activation_params.get("alpha", 1.0) != 1.0:
            raise NotImplementedError("sel: residual units are fused with ELU(alpha=1)")
        self.activation = getattr(nn, nonlinear_activation)(**nonlinear_activation_params)
        self.conv1 = NonCausalConv1d(in_channels=in_channels, out_channels=out_channels,
                                     kernel_size=kernel_size, stride=1, dilation=dilation, bias=bias)
        self.conv2 = Conv1d1x1(out_channels, out_channels, bias)

    def forward(self, x):
        """x + conv2(ELU(conv1(ELU(x)))) (:43-46) with conv1's symmetric pad
        (k-1)//2*d: the same fused op as the causal unit, whose descriptor takes
        the pad (the ELUs in the conv prologues, the residual in the 1x1's epilogue)."""
        return _fused(self, x, self.conv1.conv.padding[0])


def _fused(ru, x, pad):
    xc = CO.to_cl(x)
    dt = CO.compute_dtype()
    if xc.dtype != dt:
        xc = CO.cast(xc, dt)
    c1, c2 = ru.conv1.conv, ru.conv2
    y = CO.ResidualUnitFn.apply(xc, c1.weight, c1.bias, c2.weight, c2.bias, c1.dilation[0], pad)
    return y.transpose(1, 2)


class CausalResidualUnit(NonCausalResidualUnit):
    def __init__(self, in_channels, out_channels, kernel_size=7, dilation=1, bias=False,
                 nonlinear_activation="ELU", nonlinear_activation_params={}):
        super().__init__(in_channels=in_channels, out_channels=out_channels, kernel_size=kernel_size,
                         dilation=dilation, bias=bias, nonlinear_activation=nonlinear_activation,
                         nonlinear_activation_params=nonlinear_activation_params)
        self.conv1 = CausalConv1d(in_channels=in_channels, out_channels=out_channels,
                                  kernel_size=kernel_size, stride=1, dilation=dilation, bias=bias)

    def forward(self, x):
        return _fused(self, x, self.conv1.pad_length)

    @torch.no_grad()
    def inference(self, x):
        """Streaming step (residual_unit.py:78-81): conv1 carries its pad_buffer."""
        y = self.conv1.inference(self.activation(x))
        return x + self.conv2(self.activation(y))
