"""Vector quantizer — drop-in for the reference ``layers/vq_module.py``.

VectorQuantize (:19-104) and ResidualVQ (:107-161) keep their constructor
arguments and buffers (``embed`` (dim, n_embed), ``cluster_size``,
``embed_avg``), so reference checkpoints load.  Eval-mode forward (the denoise
trainer's, trainer/denoise.py:60) runs the fused all-stage HIP kernel
(sel/vqops.py); training mode additionally applies the EMA codebook update
(:74-80) on device after the same kernel's assignment.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from sel.vqops import ResidualVQFn


class VectorQuantize(nn.Module):
    """Vector quantization w/ exponential moving averages (EMA)."""

    def __init__(self, dim, codebook_size, decay=0.8, commitment=1.0, eps=1e-5, n_embed=None):
        super().__init__()
        n_embed = codebook_size if n_embed is None else n_embed
        self.dim = dim
        self.n_embed = n_embed
        self.decay = decay
        self.eps = eps
        self.commitment = commitment
        embed = torch.randn(dim, n_embed)
        self.register_buffer("embed", embed)
        self.register_buffer("cluster_size", torch.zeros(n_embed))
        self.register_buffer("embed_avg", embed.clone())
        # bumped by every codebook write this module makes or sees (EMA update,
        # load_state_dict, .to()/.cuda()); ResidualVQ's stack cache keys on it.
        # A write that bypasses both (.data / raw device pointers) must call
        # invalidate_codebook().
        self._codebook_epoch = 0

    def invalidate_codebook(self):
        self._codebook_epoch += 1

    def _apply(self, fn, *args, **kwargs):
        self._codebook_epoch += 1
        return super()._apply(fn, *args, **kwargs)

    def _load_from_state_dict(self, *args, **kwargs):
        self._codebook_epoch += 1
        return super()._load_from_state_dict(*args, **kwargs)

    @property
    def codebook(self):
        return self.embed.transpose(0, 1)

    def _ema(self, flatten, ind):
        """vq_module.py:74-80 (training mode only)."""
        with torch.no_grad():
            onehot_sum = torch.bincount(ind, minlength=self.n_embed).to(flatten.dtype)
            self.cluster_size.mul_(self.decay).add_(onehot_sum, alpha=1 - self.decay)
            embed_sum = torch.zeros_like(self.embed_avg).index_add_(1, ind, flatten.t())
            self.embed_avg.mul_(self.decay).add_(embed_sum, alpha=1 - self.decay)
            n = self.cluster_size.sum()
            cs = (self.cluster_size + self.eps) / (n + self.n_embed * self.eps) * n
            self.embed.copy_(self.embed_avg / cs.unsqueeze(0))
        self._codebook_epoch += 1

    def forward(self, input):
        flatten = input.reshape(-1, self.dim)
        if self.training:
            # assignment uses the pre-update codebook (reference order :64-80)
            out, loss, ppl, idx = ResidualVQFn.apply(flatten.detach(), self.embed.unsqueeze(0),
                                                     self.commitment)
            self._ema(flatten.detach().float(), idx[0])
            q = out.view_as(input)
            loss = F.mse_loss(q.detach(), input) * self.commitment
            return input + (q - input).detach(), loss, ppl[0]
        out, loss, ppl, _ = ResidualVQFn.apply(flatten, self.embed.unsqueeze(0), self.commitment)
        return out.view_as(input), loss[0], ppl[0]

    def forward_index(self, input):
        flatten = input.reshape(-1, self.dim)
        out, _, _, idx = ResidualVQFn.apply(flatten, self.embed.unsqueeze(0), self.commitment)
        return out.view_as(input), idx[0].view(*input.shape[:-1])


class ResidualVQ(nn.Module):
    """Residual VQ (https://arxiv.org/pdf/2107.03312.pdf algorithm 1)."""

    def __init__(self, *, num_quantizers, **kwargs):
        super().__init__()
        self.layers = nn.ModuleList([VectorQuantize(**kwargs) for _ in range(num_quantizers)])

    def _stacked(self):
        # the (S, D, K) codebook stack, rebuilt only when a codebook changed
        # (EMA update, load_state_dict, .to(): a bumped epoch, new storage or
        # a bumped version; writes through .data or raw pointers must call
        # VectorQuantize.invalidate_codebook())
        embeds = [l.embed for l in self.layers]
        if any(e.requires_grad for e in embeds):
            return torch.stack(embeds)
        key = tuple((l._codebook_epoch, e.data_ptr(), e._version, e.dtype, e.device)
                    for l, e in zip(self.layers, embeds))
        if getattr(self, "_stack_key", None) != key:
            self._stack_cache = torch.stack(embeds)
            self._stack_key = key
        return self._stack_cache

    def forward(self, x):
        if any(l.training for l in self.layers):
            out, residual, losses, ppls = 0.0, x, [], []
            for layer in self.layers:
                q, l_, p_ = layer(residual)
                residual = residual - q
                out = out + q
                losses.append(l_)
                ppls.append(p_)
            return out, torch.stack(losses), torch.stack(ppls)
        flatten = x.reshape(-1, x.shape[-1])
        out, losses, ppls, _ = ResidualVQFn.apply(flatten, self._stacked(), self.layers[0].commitment)
        return out.view(x.shape), losses, ppls

    def forward_index(self, x, flatten_idx=False):
        flatten = x.reshape(-1, x.shape[-1])
        out, _, _, idx = ResidualVQFn.apply(flatten, self._stacked(), self.layers[0].commitment)
        idx = idx.view(len(self.layers), *x.shape[:-1])
        if flatten_idx:
            idx = idx + (self.codebook_size * torch.arange(len(self.layers), device=idx.device)).view(
                -1, *([1] * (idx.dim() - 1)))
        return out.view(x.shape), idx.squeeze(1)

    def initial(self):
        self.codebook = torch.stack([l.codebook for l in self.layers])
        self.codebook_size = self.codebook.size(1)
        self.codebook = self.codebook.reshape(-1, self.codebook.size(-1))

    def lookup(self, indices):
        return torch.sum(F.embedding(indices, self.codebook), dim=0, keepdim=True)
