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
    """1D noncausal convolution w/ 2-sides padding (conv_layer.py:26-65).

    Only the stride-1, groups-1, symmetric-padding form is lowered to the HIP
    primitive (the shipped configs are all mode 'causal')."""

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

    def forward(self, x):
        c = self.conv
        if c.stride[0] != 1 or c.groups != 1 or 2 * c.padding[0] != (c.kernel_size[0] - 1) * c.dilation[0]:
            raise NotImplementedError("sel: NonCausalConv1d is lowered for stride 1 / 'same' padding only")
        xc = CO.to_cl(x)
        dt = CO.compute_dtype()
        if xc.dtype != dt:
            xc = CO.cast(xc, dt)
        y = _NonCausalFn.apply(xc, c.weight, c.bias, c.dilation[0], c.padding[0])
        return y.transpose(1, 2)


class _NonCausalFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, dil, pad):
        B, T, C = x.shape
        N, _, K = w.shape
        d = CO.ConvDesc(B * T, T, C, N, K, dil, pad, CO.PAD_ZERO, 0, N if b is not None else 0)
        wp = CO.pack(CO.PACK_FWD, w, 1, x.dtype)
        y = CO.prim(d, x, wp, bias=b.detach().float().contiguous() if b is not None else None)
        ctx.save_for_backward(x, wp)
        ctx.meta = (d, tuple(w.shape), b is not None)
        return y.view(B, T, N)

    @staticmethod
    def backward(ctx, gy):
        x, wp = ctx.saved_tensors
        d, ws, hb = ctx.meta
        gy = gy.contiguous()
        if gy.dtype != x.dtype:
            gy = CO.cast(gy, x.dtype)
        gx = CO.prim(d.adjoint(), gy, CO.pack_dgrad(wp)).view(x.shape) if ctx.needs_input_grad[0] else None
        gw = gb = None
        if ctx.needs_input_grad[1] or ctx.needs_input_grad[2]:
            gwp, gb = CO.wgrad(d, gy, x, hb and ctx.needs_input_grad[2])
            gw = CO.unpack(CO.PACK_FWD, gwp, ws, 1)
        return gx, gw, gb, None, None


class NonCausalConvTranspose1d(nn.Module):
    """1D noncausal transpose convolution (conv_layer.py:68-106); parameters only —
    the shipped configs use the causal variant."""

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
        raise NotImplementedError("sel: NonCausalConvTranspose1d is not on the causal hot path")


class CausalConv1d(NonCausalConv1d):
    """1D causal convolution w/ 1-side padding (conv_layer.py:109-150)."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, dilation=1, groups=1, bias=True,
                 pad_buffer=None):
        super().__init__(in_channels=in_channels, out_channels=out_channels, kernel_size=kernel_size,
                         stride=stride, padding=0, dilation=dilation, groups=groups, bias=bias)
        if groups != 1:
            raise NotImplementedError("sel: grouped CausalConv1d is not on the AudioDec hot path")
        self.stride = stride
        self.pad_length = (kernel_size - 1) * dilation
        if pad_buffer is None:
            pad_buffer = torch.zeros(1, in_channels, self.pad_length)
        self.register_buffer("pad_buffer", pad_buffer)
        # fp32 output under bf16 compute (set on a model's last layer, whose
        # output feeds the fp32 losses: no separate cast launch)
        self.out_float = False

    def forward(self, x):
        return _run_layer(x, self.conv.weight, self.conv.bias, CO.PACK_FWD, self.stride, self.dilation,
                          self.out_float)

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
        if s == 1:
            return self.forward(xb)[:, :, self.pad_length:]
        if self.pad_length != 2 * s - 1:
            raise NotImplementedError("sel: streaming strided CausalConv1d is lowered for kernel_size == 2*stride")
        xz = torch.cat((xb.new_zeros(xb.shape[0], xb.shape[1], 1), xb), -1)
        return self.forward(xz)[:, :, 2:]

    def reset_buffer(self):
        self.pad_buffer.zero_()


class CausalConvTranspose1d(NonCausalConvTranspose1d):
    """1D causal transpose convolution (conv_layer.py:153-191): replicate-pad 1,
    ConvTranspose1d(k=2s, s), crop [s:-s]; lowered to a 2-tap conv producing
    s output phases per input step."""

    def __init__(self, in_channels, out_channels, kernel_size, stride, bias=True, pad_buffer=None):
        super().__init__(in_channels=in_channels, out_channels=out_channels, kernel_size=kernel_size,
                         stride=stride, padding=0, output_padding=0, bias=bias)
        if kernel_size != 2 * stride:
            raise NotImplementedError("sel: CausalConvTranspose1d is lowered for kernel_size == 2*stride")
        self.stride = stride
        self.pad_length = 1
        if pad_buffer is None:
            pad_buffer = torch.zeros(1, in_channels, self.pad_length)
        self.register_buffer("pad_buffer", pad_buffer)

    def forward(self, x):
        return _run_layer(x, self.deconv.weight, self.deconv.bias, CO.PACK_CONVT, self.stride, 1)

    @torch.no_grad()
    def inference(self, x):
        """Streaming step (conv_layer.py:185-188): deconv(cat(pad_buffer, x))[s:-s].
        The forward kernel replicates its input's first sample in front, so
        forward(cat(buffer, x))[..., s:] is exactly that (the duplicated leading
        sample only reaches the s outputs that are dropped)."""
        xb = torch.cat((self.pad_buffer.to(x.dtype).expand(x.shape[0], -1, -1), x), -1)
        self.pad_buffer = xb[:, :, -self.pad_length:].contiguous()
        return self.forward(xb)[:, :, self.stride:]

    def reset_buffer(self):
        self.pad_buffer.zero_()
