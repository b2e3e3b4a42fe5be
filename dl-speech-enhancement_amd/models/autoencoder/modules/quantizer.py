"""Quantizer — drop-in for models/autoencoder/modules/quantizer.py (:15-48)."""
import torch

from layers.vq_module import ResidualVQ


class Quantizer(torch.nn.Module):
    def __init__(self, code_dim, codebook_num, codebook_size, model="residual_vq"):
        super().__init__()
        if model != "residual_vq":
            raise NotImplementedError(f"Model ({model}) is not supported!")
        self.codebook = ResidualVQ(dim=code_dim, num_quantizers=codebook_num, codebook_size=codebook_size)

    def initial(self):
        self.codebook.initial()

    def forward(self, z):
        zq, vqloss, perplexity = self.codebook(z.transpose(2, 1))
        return zq.transpose(2, 1), vqloss, perplexity

    def inference(self, z):
        zq, indices = self.codebook.forward_index(z.transpose(2, 1))
        return zq.transpose(2, 1), indices

    def encode(self, z):
        return self.codebook.forward_index(z.transpose(2, 1), flatten_idx=True)

    def decode(self, indices):
        return self.codebook.lookup(indices)
