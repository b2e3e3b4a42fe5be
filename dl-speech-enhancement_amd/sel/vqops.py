"""Autograd op over the residual-VQ kernel (layers/vq_module.py:61-88, :119-134)."""
import torch

from . import _lib as L


class ResidualVQFn(torch.autograd.Function):
    """(x (N, D), embeds (S, D, K)) -> (out (N, D), losses (S,), ppls (S,), idx (S, N))."""

    @staticmethod
    def forward(ctx, x, embeds, commitment):
        L.need_device(x, embeds)
        x = x.contiguous().float()
        embeds = embeds.contiguous()
        N, D = x.shape
        S, _, K = embeds.shape
        dev = x.device
        out = torch.empty_like(x)
        idx = torch.empty((S, N), dtype=torch.int64, device=dev)
        counts = torch.empty((S, K), dtype=torch.int32, device=dev)
        sqerr = torch.empty(S, dtype=torch.float64, device=dev)
        ws = L.workspace(L.lib().sel_rvq_workspace(N, S, K), dev)
        L.call("sel_rvq_fwd", L.ptr(x), N, D, L.ptr(embeds), S, K, L.ptr(out), L.ptr(idx), L.ptr(counts),
               L.ptr(sqerr), L.ptr(ws), ws.numel(), L.stream())
        loss = torch.empty(S, dtype=torch.float32, device=dev)
        ppl = torch.empty(S, dtype=torch.float32, device=dev)
        L.call("sel_rvq_finish", L.ptr(counts), L.ptr(sqerr), N, D, S, K, float(commitment), L.ptr(loss),
               L.ptr(ppl), L.stream())
        ctx.save_for_backward(x, embeds, idx)
        ctx.commitment = float(commitment)
        ctx.mark_non_differentiable(ppl, idx)
        # the perplexities / indices (and an unused loss) take no gradient:
        # None in backward instead of materialised zero tensors (two fill
        # launches per step)
        ctx.set_materialize_grads(False)
        ctx.counts = counts
        return out, loss, ppl, idx

    @staticmethod
    def backward(ctx, g_out, g_loss, g_ppl, g_idx):
        x, embeds, idx = ctx.saved_tensors
        N, D = x.shape
        K = embeds.shape[2]
        gx = torch.empty_like(x)
        go = g_out.contiguous() if g_out is not None else None
        gl = g_loss.contiguous() if g_loss is not None else None
        L.call("sel_rvq_bwd", L.ptr(x), N, D, L.ptr(embeds[0]), K, L.ptr(idx[0]), L.ptr(go), L.ptr(gl),
               ctx.commitment, L.ptr(gx), L.stream())
        return gx, None, None
