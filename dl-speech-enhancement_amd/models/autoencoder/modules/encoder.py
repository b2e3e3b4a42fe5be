"""AudioDec encoder — drop-in for models/autoencoder/modules/encoder.py (:24-123)."""
import torch

from layers.conv_layer import CausalConv1d, NonCausalConv1d
from models.autoencoder.modules.residual_unit import CausalResidualUnit, NonCausalResidualUnit

_KINDS = {"causal": (CausalResidualUnit, CausalConv1d), "noncausal": (NonCausalResidualUnit, NonCausalConv1d)}


def _check_causal(mode, name):
    """models/utils.py check_mode: streaming methods exist for the causal mode only."""
    if mode != "causal":
        raise NotImplementedError(f"{name} is not supported in {mode} mode (causal only)")


def _kinds(mode):
    if mode not in _KINDS:
        raise NotImplementedError(f"Mode ({mode}) is not supported!")
    return _KINDS[mode]


class EncoderBlock(torch.nn.Module):
    """3 residual units (dilations 1, 3, 9) then a stride-s conv with kernel 2s."""

    def __init__(self, in_channels, out_channels, stride, dilations=(1, 3, 9), bias=True, mode="causal"):
        super().__init__()
        self.mode = mode
        RU, Conv = _kinds(mode)
        self.res_units = torch.nn.ModuleList([RU(in_channels, in_channels, dilation=d) for d in dilations])
        self.num_res = len(self.res_units)
        self.conv = Conv(in_channels=in_channels, out_channels=out_channels, kernel_size=2 * stride,
                         stride=stride, bias=bias)

    def forward(self, x):
        for ru in self.res_units:
            x = ru(x)
        return self.conv(x)

    def inference(self, x):
        _check_causal(self.mode, "inference")
        for ru in self.res_units:
            x = ru.inference(x)
        return self.conv.inference(x)


class Encoder(torch.nn.Module):
    def __init__(self, input_channels, encode_channels, channel_ratios=(2, 4, 8, 16), strides=(3, 4, 5, 5),
                 kernel_size=7, bias=True, mode="causal"):
        super().__init__()
        assert len(channel_ratios) == len(strides)
        self.mode = mode
        _, Conv = _kinds(mode)
        self.conv = Conv(in_channels=input_channels, out_channels=encode_channels, kernel_size=kernel_size,
                         stride=1, bias=False)
        self.conv_blocks = torch.nn.ModuleList()
        cin = encode_channels
        for ratio, stride in zip(channel_ratios, strides):
            cout = encode_channels * ratio
            self.conv_blocks.append(EncoderBlock(cin, cout, stride, bias=bias, mode=mode))
            cin = cout
        self.num_blocks = len(self.conv_blocks)
        self.out_channels = cin

    def forward(self, x):
        x = self.conv(x)
        for blk in self.conv_blocks:
            x = blk(x)
        return x

    def encode(self, x):
        """Streaming encoder step (encoder.py:118-123)."""
        _check_causal(self.mode, "encode")
        x = self.conv.inference(x)
        for blk in self.conv_blocks:
            x = blk.inference(x)
        return x
