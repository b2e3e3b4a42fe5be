"""Projector — drop-in for models/autoencoder/modules/projector.py (:20-56)."""
import torch

from layers.conv_layer import CausalConv1d, NonCausalConv1d
from sel.bnops import BatchNorm1d


class Projector(torch.nn.Module):
    def __init__(self, input_channels, code_dim, kernel_size=3, stride=1, bias=False, mode="causal",
                 model="conv1d"):
        super().__init__()
        self.mode = mode
        Conv = {"causal": CausalConv1d, "noncausal": NonCausalConv1d}.get(mode)
        if Conv is None:
            raise NotImplementedError(f"Mode ({mode}) is not supported!")
        if model == "conv1d":
            self.project = Conv(input_channels, code_dim, kernel_size=kernel_size, stride=stride, bias=bias)
        elif model == "conv1d_bn":   # (:40-44) the conv, then BatchNorm1d on the HIP kernels (sel.bnops)
            self.project = torch.nn.Sequential(
                Conv(input_channels, code_dim, kernel_size=kernel_size, stride=stride, bias=bias),
                BatchNorm1d(code_dim))
        else:
            raise NotImplementedError(f"Model ({model}) is not supported!")

    def forward(self, x):
        return self.project(x)

    def encode(self, x):
        """Streaming step (projector.py:52-54)."""
        if self.mode != "causal":
            raise NotImplementedError(f"encode is not supported in {self.mode} mode (causal only)")
        return self.project.inference(x)
