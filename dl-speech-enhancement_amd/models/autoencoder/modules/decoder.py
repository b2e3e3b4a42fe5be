"""AudioDec decoder — drop-in for models/autoencoder/modules/decoder.py (:24-128)."""
import torch

from layers.conv_layer import CausalConv1d, CausalConvTranspose1d, NonCausalConv1d, NonCausalConvTranspose1d
from models.autoencoder.modules.residual_unit import CausalResidualUnit, NonCausalResidualUnit

_KINDS = {"causal": (CausalResidualUnit, CausalConvTranspose1d, CausalConv1d),
          "noncausal": (NonCausalResidualUnit, NonCausalConvTranspose1d, NonCausalConv1d)}


def _check_causal(mode, name):
    """models/utils.py check_mode: streaming methods exist for the causal mode only."""
    if mode != "causal":
        raise NotImplementedError(f"{name} is not supported in {mode} mode (causal only)")


def _kinds(mode):
    if mode not in _KINDS:
        raise NotImplementedError(f"Mode ({mode}) is not supported!")
    return _KINDS[mode]


class DecoderBlock(torch.nn.Module):
    """Transposed conv (kernel 2s, stride s) then 3 residual units."""

    def __init__(self, in_channels, out_channels, stride, dilations=(1, 3, 9), bias=True, mode="causal"):
        super().__init__()
        self.mode = mode
        RU, ConvT, _ = _kinds(mode)
        self.conv = ConvT(in_channels=in_channels, out_channels=out_channels, kernel_size=2 * stride,
                          stride=stride, bias=bias)
        self.res_units = torch.nn.ModuleList([RU(out_channels, out_channels, dilation=d) for d in dilations])
        self.num_res = len(self.res_units)

    def forward(self, x):
        x = self.conv(x)
        for ru in self.res_units:
            x = ru(x)
        return x

    def inference(self, x):
        _check_causal(self.mode, "inference")
        x = self.conv.inference(x)
        for ru in self.res_units:
            x = ru.inference(x)
        return x


class Decoder(torch.nn.Module):
    # set by models/autoencoder_without_PQC: the bottleneck conv1 is constructed but skipped
    skip_conv1 = False

    def __init__(self, code_dim, output_channels, decode_channels, channel_ratios=(16, 8, 4, 2),
                 strides=(5, 5, 4, 3), kernel_size=7, bias=True, mode="causal"):
        super().__init__()
        assert len(channel_ratios) == len(strides)
        self.mode = mode
        _, _, Conv = _kinds(mode)
        self.conv1 = Conv(in_channels=code_dim, out_channels=decode_channels * channel_ratios[0],
                          kernel_size=kernel_size, stride=1, bias=False)
        self.conv_blocks = torch.nn.ModuleList()
        for i, stride in enumerate(strides):
            cin = decode_channels * channel_ratios[i]
            cout = decode_channels * channel_ratios[i + 1] if i < len(channel_ratios) - 1 else decode_channels
            self.conv_blocks.append(DecoderBlock(cin, cout, stride, bias=bias, mode=mode))
        self.num_blocks = len(self.conv_blocks)
        self.conv2 = Conv(cout, output_channels, kernel_size, 1, bias=False)
        # the waveform leaves in fp32 (the losses' dtype) straight from the
        # conv epilogue, where AudioDec.py's y.float() would cast it
        self.conv2.out_float = True

    def forward(self, z):
        x = z if self.skip_conv1 else self.conv1(z)
        for blk in self.conv_blocks:
            x = blk(x)
        return self.conv2(x)

    def decode(self, z):
        """Streaming decoder step (decoder.py:123-128)."""
        _check_causal(self.mode, "decode")
        x = z if self.skip_conv1 else self.conv1.inference(z)
        for blk in self.conv_blocks:
            x = blk.inference(x)
        return self.conv2.inference(x)
