"""Convolution layers — drop-in for the reference ``layers/conv_layer.py``.

Same classes, constructor arguments, sub-module names and ``state_dict`` keys
(``conv.weight``/``conv.bias``/``pad_buffer``, ``deconv.*``), so reference
checkpoints load unchanged.  ``forward`` runs the HIP conv primitive
(sel/convops.py) on channels-last activations: inputs/outputs keep the
reference's (B, C, T) shape, physically stored as (B, T, C).
"""
import torch
import torch.nn as nn

from sel import convops as CO
from sel import genconv as GC


def _run_layer(x, weight, bias, kind, stride, dilation, out_float=False):
    """(B, C, T) in -> (B, C', T') out through ConvLayerFn, in the active precision
    (out_float: fp32 output whatever the compute dtype)."""
    xc = CO.to_cl(x)
    dt = CO.compute_dtype()
    if xc.dtype != dt:
        xc = CO.cast(xc, dt)
    if out_float and dt != torch.float32:
        y = CO.ConvLayerFn.apply(xc, weight, bias, kind, stride, dilation, True)
    else:
        y = CO.ConvLayerFn.apply(xc, weight, bias, kind, stride, dilation)
    return y.transpose(1, 2)


class Conv1d1x1(nn.Conv1d):
    """1x1 Conv1d (conv_layer.py:19-23)."""

    def __init__(self, in_channels, out_channels, bias=True):
        super().__init__(in_channels, out_channels, kernel_size=1, bias=bias)

    def forward(self, x):
        return _run_layer(x, self.weight, self.bias, CO.PACK_FWD, 1, 1)


class NonCausalConv1d(nn.Module):
    """1D noncausal convolution w/ 2-sides padding (conv_layer.py:26-65): any
    stride, padding, dilation and groups (sel.genconv lowers them onto the
    stride-1 HIP primitive; the stride-1 'same' form is a single launch)."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=-1, dilation=1,
                 groups=1, bias=True):
        super().__init__()
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.kernel_size = kernel_size
        if padding < 0:
            padding = (kernel_size - 1) // 2 * dilation
        self.dilation = dilation
        self.conv = nn.Conv1d(in_channels=in_channels, out_channels=out_channels, kernel_size=kernel_size,
                              stride=stride, padding=padding, dilation=dilation, groups=groups, bias=bias)
        self.out_float = False   # fp32 output under bf16 compute (see CausalConv1d)

    def forward(self, x):
        c = self.conv
        y = _general(x, lambda xc: GC.conv1d(xc, c.weight, c.bias, c.stride[0], c.padding[0], c.dilation[0],
                                              c.groups))
        return CO.cast(y, torch.float32) if self.out_float else y


def _general(x, fn):
    """(B, C, T) -> fn(channels-last x in the compute dtype) -> (B, C', T')."""
    xc = CO.to_cl(x)
    dt = CO.compute_dtype()
    if xc.dtype != dt:
        xc = CO.cast(xc, dt)
    return fn(xc).transpose(1, 2)


class NonCausalConvTranspose1d(nn.Module):
    """1D noncausal transpose convolution (conv_layer.py:68-106): any stride,
    padding, output_padding and groups (sel.genconv: one primitive launch
    producing the stride's output phases per input row)."""

    def __init__(self, in_channels, out_channels, kernel_size, stride, padding=-1, output_padding=-1,
                 groups=1, bias=True):
        super().__init__()
        if padding < 0:
            padding = (stride + 1) // 2
        if output_padding < 0:
            output_padding = 1 if stride % 2 else 0
        self.deconv = nn.ConvTranspose1d(in_channels=in_channels, out_channels=out_channels,
                                         kernel_size=kernel_size, stride=stride, padding=padding,
                                         output_padding=output_padding, groups=groups, bias=bias)

    def forward(self, x):
        d = self.deconv
        return _general(x, lambda xc: GC.conv_transpose1d(xc, d.weight, d.bias, d.stride[0], d.padding[0],
                                                           d.output_padding[0], d.groups))


class CausalConv1d(NonCausalConv1d):
    """1D causal convolution w/ 1-side padding (conv_layer.py:109-150)."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, dilation=1, groups=1, bias=True,
                 pad_buffer=None):
        super().__init__(in_channels=in_channels, out_channels=out_channels, kernel_size=kernel_size,
                         stride=stride, padding=0, dilation=dilation, groups=groups, bias=bias)
        self.stride = stride
        self.pad_length = (kernel_size - 1) * dilation
        if pad_buffer is None:
            pad_buffer = torch.zeros(1, in_channels, self.pad_length)
        self.register_buffer("pad_buffer", pad_buffer)
        # fp32 output under bf16 compute (set on a model's last layer, whose
        # output feeds the fp32 losses: no separate cast launch)
        self.out_float = False

    def _packed_form(self, T):
        """The dedicated ConvLayerFn packing applies (ungrouped; stride 1, or
        the k = 2s downsampling conv on a stride-aligned input)?"""
        s = self.stride
        return self.conv.groups == 1 and (s == 1 or (self.kernel_size == 2 * s and T % s == 0))

    def forward(self, x):
        if self._packed_form(x.shape[-1]):
            return _run_layer(x, self.conv.weight, self.conv.bias, CO.PACK_FWD, self.stride, self.dilation,
                              self.out_float)
        # grouped / other strides (sel.genconv): left pad (k-1)*d, T_out = ceil(T / s)
        c = self.conv
        y = _general(x, lambda xc: GC.conv1d(xc, c.weight, c.bias, self.stride, self.pad_length, self.dilation,
                                              c.groups, (x.shape[-1] - 1) // self.stride + 1))
        return CO.cast(y, torch.float32) if self.out_float else y

    @torch.no_grad()
    def inference(self, x):
        """Streaming step (conv_layer.py:144-147): conv over cat(pad_buffer, x),
        keeping the last pad_length input samples.  Runs the causal forward kernel
        on a shifted input: with its own (K-1)d zero pad in front,
        forward(cat(0^j, buffer, x))[..., m:] equals the valid conv of
        cat(buffer, x), where j = 0 and m = pad_length / stride for stride 1, and
        j = 1, m = 2 for the kernel-2s stride-s downsampling convs."""
        xb = torch.cat((self.pad_buffer.to(x.dtype).expand(x.shape[0], -1, -1), x), -1)
        if self.pad_length == 0:
            # kernel 1: the reference keeps x[:, :, -0:], i.e. the whole
            # concatenated input, and returns the conv over all of it
            self.pad_buffer = xb.contiguous()
            return self.forward(xb)
        self.pad_buffer = xb[:, :, -self.pad_length:].contiguous()
        s = self.stride
        c = self.conv
        if c.groups != 1 or (s > 1 and self.kernel_size != 2 * s):
            # the valid conv of cat(buffer, x) (sel.genconv, no padding)
            return _general(xb, lambda xc: GC.conv1d(xc, c.weight, c.bias, s, 0, self.dilation, c.groups))
        if s == 1:
            return self.forward(xb)[:, :, self.pad_length:]
        xz = torch.cat((xb.new_zeros(xb.shape[0], xb.shape[1], 1), xb), -1)
        return self.forward(xz)[:, :, 2:]

    def reset_buffer(self):
        self.pad_buffer.zero_()


class CausalConvTranspose1d(NonCausalConvTranspose1d):
    """1D causal transpose convolution (conv_layer.py:153-191): replicate-pad 1,
    ConvTranspose1d(k, s), crop [s:-s].  k = 2s (every shipped config) is a
    2-tap conv producing s output phases per input step with the replicate pad
    in the kernel; other k go through sel.genconv."""

    def __init__(self, in_channels, out_channels, kernel_size, stride, bias=True, pad_buffer=None):
        super().__init__(in_channels=in_channels, out_channels=out_channels, kernel_size=kernel_size,
                         stride=stride, padding=0, output_padding=0, bias=bias)
        self.stride = stride
        self.kernel_size = kernel_size
        self.pad_length = 1
        if pad_buffer is None:
            pad_buffer = torch.zeros(1, in_channels, self.pad_length)
        self.register_buffer("pad_buffer", pad_buffer)

    def _deconv_cropped(self, x):
        """deconv(x)[:, :, s:-s] through sel.genconv (any kernel size)."""
        d, s = self.deconv, self.stride
        L = (x.shape[-1] - 1) * s + self.kernel_size - 2 * s
        return _general(x, lambda xc: GC.conv_transpose1d(xc, d.weight, d.bias, s, s, 0, 1, L))

    def forward(self, x):
        if self.kernel_size == 2 * self.stride:
            return _run_layer(x, self.deconv.weight, self.deconv.bias, CO.PACK_CONVT, self.stride, 1)
        return self._deconv_cropped(torch.cat((x[:, :, :1], x), -1))

    @torch.no_grad()
    def inference(self, x):
        """Streaming step (conv_layer.py:185-188): deconv(cat(pad_buffer, x))[s:-s].
        The forward kernel replicates its input's first sample in front, so
        forward(cat(buffer, x))[..., s:] is exactly that (the duplicated leading
        sample only reaches the s outputs that are dropped)."""
        xb = torch.cat((self.pad_buffer.to(x.dtype).expand(x.shape[0], -1, -1), x), -1)
        self.pad_buffer = xb[:, :, -self.pad_length:].contiguous()
        if self.kernel_size != 2 * self.stride:
            return self._deconv_cropped(xb)
        return self.forward(xb)[:, :, self.stride:]

    def reset_buffer(self):
        self.pad_buffer.zero_()
