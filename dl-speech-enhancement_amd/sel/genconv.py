"""General Conv1d / ConvTranspose1d lowered onto the stride-1 conv primitive.

The AudioDec causal hot path has dedicated packings (sel.convops.ConvLayerFn:
the k = 2s strided conv, the k = 2s transposed conv).  The reference's layer
classes also accept any stride, padding, dilation, groups and output_padding
(layers/conv_layer.py:26-106, :109-191) and the noncausal AudioDec mode uses
them (encoder.py:38-57, decoder.py:38-57: NonCausalConv1d(k = 2s, stride s,
padding s - 1), NonCausalConvTranspose1d(k = 2s, stride s, padding (s+1)//2,
output_padding s % 2)).  Every such layer is one launch of the same HIP
primitive (sel_conv_fwd: y[r] = b + sum_k W[k] x[r + k*dil - pad] within each
sequence, zero outside), reached by re-indexing only:

* stride s: the input is folded into phases, x'[u, j*C + c] = x[u*s + j, c], so
  tap k (offset o_k = k*dil - pad) becomes row offset floor(o_k / s) of phase
  o_k mod s: a stride-1 conv with ceil-span taps over s*C channels;
* transposed stride s: output phase j of row u is sum_m W[:, :, j + m*s]^T
  x[u - m], i.e. a causal stride-1 conv producing s*C_out channels per row,
  unfolded to s rows and cropped by the padding;
* groups: the block-diagonal dense weight (the shipped configs have none; a
  grouped layer costs `groups` times its flops here, the discriminator's grouped
  kernels in sel.dconvops are the fast form);
* padding beyond the primitive's range: explicit zero rows (left pad beyond the
  receptive field, right rows for longer outputs), then a crop.

Weight re-indexing is differentiable torch view/index work on the (small)
parameters; every activation-sized multiply-add, its adjoint and its weight
gradient run in the HIP kernels.  The weight gradient of a layer with more than
8 taps (the primitive's wgrad tile bound) is assembled from tap groups of at
most 8, each against the input shifted by its group's offset.
"""
import torch
import torch.nn.functional as F

from . import convops as CO

_WG_TAPS = 8   # sel_conv_wgrad: K <= 8 (conv.hip wgrad_impl)


class Stride1Fn(torch.autograd.Function):
    """y[b, t, n] = bias[n] + sum_{k, c} w[n, c, k] x[b, t + k*dil - pad, c]
    (x zero outside [0, T)), t in [0, T): one sel_conv_fwd launch; x (B, T, C)
    contiguous in the compute dtype, w (N, C, K) fp32 (any autograd history),
    0 <= pad <= (K-1)*dil so the adjoint is the same primitive."""

    @staticmethod
    def forward(ctx, x, w, b, dil, pad):
        B, T, C = x.shape
        N, _, K = w.shape
        if not 0 <= pad <= (K - 1) * dil:
            raise ValueError(f"Stride1Fn: pad {pad} outside [0, {(K - 1) * dil}]")
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
        want_b = hb and ctx.needs_input_grad[2]
        if ctx.needs_input_grad[1] or want_b:
            gw, gb = _wgrad(d, gy, x, ws, want_b)
        return gx, gw, gb, None, None


def _wgrad(d, gy, x, ws, want_b):
    """Weight (torch layout (N, C, K), fp32) and bias gradient of Stride1Fn."""
    N, C, K = ws
    if K <= _WG_TAPS:
        gwp, gb = CO.wgrad(d.with_(bias_period=N if want_b else 0), gy, x, want_b)
        return CO.unpack(CO.PACK_FWD, gwp, ws, 1), gb
    B, T, _ = x.shape
    parts, gb = [], None
    for k0 in range(0, K, _WG_TAPS):
        kg = min(_WG_TAPS, K - k0)
        pg = d.pad - k0 * d.dil
        xin = x
        if pg < 0:   # taps reading ahead of the output row: the input shifted by -pg rows
            sh = -pg
            pg = 0
            xin = x.new_zeros(x.shape)
            if sh < T:
                xin[:, :T - sh] = x[:, sh:]
        bg = want_b and k0 == 0
        dg = CO.ConvDesc(d.rows, d.T, C, N, kg, d.dil, pg, CO.PAD_ZERO, 0, N if bg else 0)
        gwp, gbg = CO.wgrad(dg, gy, xin.contiguous(), bg)
        parts.append(CO.unpack(CO.PACK_FWD, gwp, (N, C, kg), 1))
        if bg:
            gb = gbg
    return torch.cat(parts, 2), gb


def _rows(x, w, b, dil, pad, T_out):
    """(B, T, C) -> (B, T_out, N): y[t] = b + sum_k w[:, :, k] x[t + k*dil - pad]."""
    B, T, C = x.shape
    K = w.shape[2]
    if T_out <= 0:
        raise ValueError(f"conv output length {T_out} <= 0 (input length {T})")
    e = max(pad - (K - 1) * dil, 0)     # left zeros beyond the primitive's pad range: same rows out
    r = max(T_out - T - e, 0)           # right zeros: outputs past the input length
    if e or r:
        x = F.pad(x, (0, 0, e, r))
    y = Stride1Fn.apply(x.contiguous(), w, b, dil, pad - e)
    return y if y.shape[1] == T_out else y[:, :T_out]


_POS = {}


def _positions(pos, device):
    """Device index tensor of the phase-fold tap positions, made once per layer
    geometry (no host-to-device copy per call: capturable in a HIP graph)."""
    key = (pos, str(device))
    t = _POS.get(key)
    if t is None:
        t = _POS[key] = torch.tensor(pos, dtype=torch.int64, device=device)
    return t


def _dense(w, groups):
    """Grouped torch weight (N, C/g, K) -> block-diagonal (N, C, K)."""
    if groups == 1:
        return w
    N, Cg, K = w.shape
    eye = torch.eye(groups, dtype=w.dtype, device=w.device)
    return (w.view(groups, N // groups, 1, Cg, K) * eye.view(groups, 1, groups, 1, 1)).reshape(N, groups * Cg, K)


def conv1d(x, w, b, stride=1, pad_left=0, dilation=1, groups=1, T_out=None):
    """torch Conv1d semantics on channels-last x (B, T, C) in the compute dtype:
    y[t] = b + sum_{k,c} w[n, c, k] x[t*stride + k*dilation - pad_left, c] for
    t < T_out (default: the symmetric-pad length of nn.Conv1d(padding=pad_left))."""
    B, T, C = x.shape
    N, Cg, K = w.shape
    if Cg * groups != C or N % groups:
        raise ValueError(f"conv1d: weight {tuple(w.shape)} / groups {groups} does not match {C} input channels")
    if T_out is None:
        T_out = (T + 2 * pad_left - dilation * (K - 1) - 1) // stride + 1
    wd = _dense(w, groups)
    s = stride
    if s == 1:
        return _rows(x, wd, b, dilation, pad_left, T_out)
    offs = [k * dilation - pad_left for k in range(K)]
    q = [o // s for o in offs]          # row offset (floor) and phase of every tap
    j = [o % s for o in offs]
    qmin, kp = min(q), max(q) - min(q) + 1
    pos = _positions(tuple((qk - qmin) * s + jk for qk, jk in zip(q, j)), w.device)
    wf = wd.new_zeros(N, kp * s, C).index_copy(1, pos, wd.permute(0, 2, 1))
    wf = wf.view(N, kp, s * C).permute(0, 2, 1)            # (N, s*C, kp)
    tf = max(-(-T // s), 1)
    if tf * s != T:
        x = F.pad(x, (0, 0, 0, tf * s - T))
    return _rows(x.reshape(B, tf, s * C), wf, b, 1, -qmin, T_out)


def conv_transpose1d(x, w, b, stride=1, padding=0, output_padding=0, groups=1, L_out=None):
    """torch ConvTranspose1d semantics (dilation 1) on channels-last x (B, T, Cin)
    with w (Cin, Cout/g, K): returns (B, L_out, Cout), L_out = (T-1)*stride -
    2*padding + K + output_padding unless given."""
    B, T, C = x.shape
    Cin, Cog, K = w.shape
    if Cin != C or Cin % groups:
        raise ValueError(f"conv_transpose1d: weight {tuple(w.shape)} / groups {groups} does not match {C} channels")
    cout = Cog * groups
    if groups > 1:
        eye = torch.eye(groups, dtype=w.dtype, device=w.device)
        w = (w.view(groups, Cin // groups, 1, Cog, K) * eye.view(groups, 1, groups, 1, 1)).reshape(Cin, cout, K)
    s = stride
    if L_out is None:
        L_out = (T - 1) * s - 2 * padding + K + output_padding
    m = -(-K // s)
    if m * s != K:
        w = F.pad(w, (0, m * s - K))
    # W'[(j, n), c, k'] = w[c, n, j + (m-1-k')*s]: phase j of output row u from x[u - (m-1-k')]
    wc = w.view(Cin, cout, m, s).permute(3, 1, 0, 2).flip(3).reshape(s * cout, Cin, m)
    U = (padding + L_out - 1) // s + 1
    bb = b.repeat(s) if b is not None else None
    z = _rows(x, wc, bb, 1, m - 1, U)
    return z.reshape(B, U * s, cout)[:, padding:padding + L_out]
