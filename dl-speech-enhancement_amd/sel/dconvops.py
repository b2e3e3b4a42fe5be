"""Autograd ops over the HiFi-GAN discriminator kernels of libsel.so (dconv.hip).

A sub-discriminator (one HiFiGANScaleDiscriminator or HiFiGANPeriodDiscriminator,
models/vocoder/modules/discriminator.py:26-372) is a chain of convs with
LeakyReLU; it runs as ONE autograd Function whose forward keeps every layer's
output in a channels-last buffer (B_seq, T_alloc, C) — T_alloc padded to the
next layer's stride so its phase view is free — and returns the reference-layout
views of them, and whose backward walks the chain with the adjoint primitive,
adding the gradients that arrive on the feature maps (feature matching) before
each LeakyReLU' multiply.

Reference layouts returned (views, no copies):
  scale discriminator:  (B, C, T)         <- buffer (B, T_alloc, C)
  period discriminator: (B, C, T/p, p)    <- buffer (B*p, L_alloc, C)
                        final (B, L*p)    (a copy, as torch.flatten in :134)
"""
import ctypes
import os
import weakref

import torch
from torch.optim.optimizer import register_optimizer_step_post_hook as _register_optimizer_step_post_hook

from . import _lib as L
from .convops import BF16, F32, _code, compute_dtype


class DConvDesc(ctypes.Structure):
    """include/sel.h sel_dconv_desc"""
    _fields_ = [(n, ctypes.c_int32) for n in ("B", "Tv", "Tvs", "ldx", "Tvo", "Tvalid", "ldo", "K", "q0", "S", "Cs",
                                               "Cg", "G", "So", "Ns", "Ng", "act")] + [("slope", ctypes.c_float)]


def geometry(Kt, stride, pad):
    K, q0 = ctypes.c_int(), ctypes.c_int()
    L.check(L.load().sel_dconv_geometry(Kt, stride, pad, ctypes.byref(K), ctypes.byref(q0)), "sel_dconv_geometry")
    return K.value, q0.value


def _roundup(v, m):
    return (v + m - 1) // m * m


# zero rows per sequence the period chain's layouts keep after the valid ones
# (>= the widest tap reach across a sequence boundary of its convs: k5, pad 2)
FLAT_GAP = 2


def period_alloc(Lv, specs, gap=FLAT_GAP):
    """Rows per folded sequence for an MPD chain on Lv valid rows such that every
    layer's phase-view input and output share one row pitch with >= gap zero
    rows after each sequence (the layout the warp-specialised kernel tiles
    across sequences: conv.hip dconv_ws_fwd).  Falls back to the plain
    roundup when the chain has a non-integer stride product."""
    T, prod = Lv, 1
    for sp in specs:
        T = sp.t_out(T)
        prod *= sp.stride
    return max(_roundup(Lv, specs[0].stride), prod * (T + gap))


def chain_layout(specs, T0, T_alloc0):
    """Per layer (T_in, T_alloc_in, T_out, T_out_alloc) of a chain on T0 valid
    of T_alloc0 allocated input rows: outputs padded to the next layer's stride,
    or — where the input pitch allows it — sharing the phase-view input's row
    pitch with >= FLAT_GAP zero rows per sequence (the period_alloc layout)."""
    out = []
    T_in, T_alloc_in = T0, T_alloc0
    for li, sp in enumerate(specs):
        T_out = sp.t_out(T_in)
        nxt = specs[li + 1].stride if li + 1 < len(specs) else 1
        T_out_alloc = _roundup(T_out, nxt)
        if T_alloc_in % sp.stride == 0 and (T_alloc_in // sp.stride) % nxt == 0 and \
                T_alloc_in // sp.stride - T_out >= FLAT_GAP:
            T_out_alloc = T_alloc_in // sp.stride
        out.append((T_in, T_alloc_in, T_out, T_out_alloc))
        T_in, T_alloc_in = T_out, T_out_alloc
    return out


class LayerSpec:
    """One conv of a sub-discriminator: torch Conv1d(cin, cout, Kt, stride,
    padding=pad, groups) (or Conv2d (Kt, 1) on the period axis), LeakyReLU after
    it when `leaky`."""

    __slots__ = ("cin", "cout", "Kt", "stride", "pad", "groups", "leaky", "K", "q0")

    def __init__(self, cin, cout, Kt, stride, pad, groups, leaky):
        self.cin, self.cout, self.Kt, self.stride, self.pad = cin, cout, Kt, stride, pad
        self.groups, self.leaky = groups, leaky
        self.K, self.q0 = geometry(Kt, stride, pad)

    def t_out(self, T):
        return (T + 2 * self.pad - self.Kt) // self.stride + 1


def _fwd_desc(sp, Bs, T_in, T_alloc_in, T_out, T_out_alloc, slope):
    """Forward layer: x (Bs, T_alloc_in rows, T_in valid; rows past T_in are
    zero) in its phase view (T_alloc_in / s rows of s * cin channels, the first
    ceil(T_in / s) of them holding samples) -> y (Bs, T_out_alloc rows, T_out
    computed, the rest written as zeros)."""
    s = sp.stride
    return DConvDesc(B=Bs, Tv=(T_in + s - 1) // s, Tvs=T_alloc_in // s, ldx=s * sp.cin, Tvo=T_out_alloc, Tvalid=T_out,
                     ldo=sp.cout, K=sp.K, q0=sp.q0, S=s, Cs=sp.cin, Cg=sp.cin // sp.groups, G=sp.groups, So=1,
                     Ns=sp.cout, Ng=sp.cout // sp.groups, act=1 if sp.leaky else 0, slope=slope)


def _dgrad_desc(sp, Bs, T_alloc_in, T_out, T_out_alloc, slope, prev_leaky, T_in=None):
    """Adjoint of the forward layer: gout (Bs, T_out_alloc rows, T_out valid, N
    channels) -> gin in the phase view of the layer input (Bs, T_alloc_in / s
    rows, s * cin channels); with T_in, phase rows past ceil(T_in / s) (no input
    sample there) are written as zeros instead of computed."""
    s = sp.stride
    Tvo = T_alloc_in // s
    Tval = Tvo if T_in is None else (T_in + s - 1) // s
    return DConvDesc(B=Bs, Tv=T_out, Tvs=T_out_alloc, ldx=sp.cout, Tvo=Tvo, Tvalid=Tval, ldo=s * sp.cin, K=sp.K,
                     q0=-sp.q0 - (sp.K - 1), S=1, Cs=sp.cout, Cg=sp.cout // sp.groups, G=sp.groups, So=s,
                     Ns=sp.cin, Ng=sp.cin // sp.groups, act=0, slope=slope)


class _DPackJob(ctypes.Structure):
    """include/sel.h sel_dpack_job"""
    _fields_ = [("w", ctypes.c_void_p), ("wg", ctypes.c_void_p), ("out", ctypes.c_void_p)] + \
        [(n, ctypes.c_int32) for n in ("mode", "N", "Cg", "Kt", "stride", "pad", "G", "reserved")]


class _DPackCache:
    """Packed forms of the discriminator weights, reused until the parameter
    changes: the version counter (copy_, load_state_dict, foreach Adam) or an
    optimizer step on it (torch's fused Adam does not bump the version; same
    global post-step hook as sel.convops.PackCache).  A D forward + adjoint
    otherwise repacks every layer at every call (3 D passes per GAN step)."""

    def __init__(self):
        self._e = {}

    def get(self, sp, w, wg, dtype, mode):
        key = (id(w), mode, dtype, sp.Kt, sp.stride, sp.pad, sp.groups)
        ver = (w._version, wg._version if wg is not None else None)
        hit = self._e.get(key)
        if hit is not None and hit[0]() is w and hit[1] == ver:
            return hit[2]
        out = _pack(sp, w, wg, dtype, mode)
        self._e[key] = (weakref.ref(w), ver, out)
        return out

    def prefetch(self, items):
        """Pack every stale (sp, w, wg, dtype, mode) of `items` in ONE
        sel_dconv_pack_many launch (per dtype) instead of one launch per layer
        and mode at first use (a GAN step repacks ~100 discriminator forms)."""
        miss = []
        for sp, w, wg, dtype, mode in items:
            key = (id(w), mode, dtype, sp.Kt, sp.stride, sp.pad, sp.groups)
            ver = (w._version, wg._version if wg is not None else None)
            hit = self._e.get(key)
            if hit is not None and hit[0]() is w and hit[1] == ver:
                continue
            miss.append((key, ver, sp, w, wg, dtype, mode))
        for dtype in dict.fromkeys(m[5] for m in miss):
            group = [m for m in miss if m[5] == dtype]
            jobs = (_DPackJob * len(group))()
            keep = []
            fresh = {}  # forward forms packed by this call: id(w) etc. -> buffer
            # forward forms first, so an adjoint form can be their transpose (mode 2)
            group.sort(key=lambda m: m[6])
            for i, (key, ver, sp, w, wg, _dt, mode) in enumerate(group):
                N, Cg = sp.cout, sp.cin // sp.groups
                out = torch.empty(N * sp.K * sp.stride * Cg, dtype=dtype, device=w.device)
                fkey = (key[0], 0) + key[2:]
                src = fresh.get(fkey)
                if mode == 1 and src is None:
                    hit = self._e.get(fkey)
                    if hit is not None and hit[0]() is w and hit[1] == ver:
                        src = hit[2]
                if mode == 1 and src is not None:
                    keep.append(src)
                    jobs[i] = _DPackJob(src.data_ptr(), None, out.data_ptr(), 2, N, Cg, sp.Kt, sp.stride, sp.pad,
                                        sp.groups, 0)
                else:
                    wc = w.detach().contiguous().float()
                    gc = wg.detach().contiguous().float() if wg is not None else None
                    keep += [wc, gc]
                    jobs[i] = _DPackJob(wc.data_ptr(), gc.data_ptr() if gc is not None else None, out.data_ptr(),
                                        mode, N, Cg, sp.Kt, sp.stride, sp.pad, sp.groups, 0)
                if mode == 0:
                    fresh[key] = out
                self._e[key] = (weakref.ref(w), ver, out)
            L.call("sel_dconv_pack_many", ctypes.cast(jobs, ctypes.c_void_p), len(group), _code(dtype), L.stream())

    def mark_stale(self, params):
        ids = {id(p) for p in params}
        for k in [k for k in self._e if k[0] in ids]:
            del self._e[k]

    def prune(self):
        for k in [k for k, v in self._e.items() if v[0]() is None]:
            del self._e[k]


DPACKS = _DPackCache()


def _optimizer_stepped(optimizer, args, kwargs):
    # (parameters without a gradient were not updated: torch's optimizers skip them)
    DPACKS.mark_stale([p for g in optimizer.param_groups for p in g["params"] if p.grad is not None])
    DPACKS.prune()


_register_optimizer_step_post_hook(_optimizer_stepped)


def pack(sp, w, wg, dtype, mode):
    """Cached packed form (see _DPackCache); weight_v's entry also tracks weight_g."""
    return DPACKS.get(sp, w, wg, dtype, mode)


def _pack(sp, w, wg, dtype, mode):
    """torch weight (or weight_v with weight_g) -> packed forward (mode 0) /
    adjoint (mode 1) form in `dtype`."""
    N, Cg = sp.cout, sp.cin // sp.groups
    nred = sp.stride * Cg
    n = N * sp.K * nred
    out = torch.empty(n, dtype=dtype, device=w.device)
    wc = w.detach().contiguous().float()
    gc = wg.detach().contiguous().float() if wg is not None else None
    L.call("sel_dconv_pack", mode, L.ptr(wc), L.ptr(gc), N, Cg, sp.Kt, sp.stride, sp.pad, sp.groups, _code(dtype),
           L.ptr(out), L.stream())
    return out


def prim(desc, x, wp, out, bias=None, aux=None, res=None, tag=""):
    L.call("sel_dconv_fwd", ctypes.byref(desc), _code(x.dtype), L.ptr(x), L.ptr(wp), L.ptr(bias), L.ptr(aux),
           L.ptr(res), L.ptr(out), L.stream(), meta=lambda: _meta(desc, x, out, tag))
    return out


PATH_NAMES = {0: "valu", 1: "mfma", 2: "short", 3: "pf", 4: "ws", 5: "ws_flat", 6: "tiny", 7: "gpf", 8: "shortx"}


def kernel(desc, dtype):
    """(path, kernel name) a sel_dconv_fwd launch of this descriptor takes
    (include/sel.h SEL_DPATH_*; the launcher's own decision, no GPU needed)."""
    buf = ctypes.create_string_buffer(96)
    path = L.load().sel_dconv_kernel(ctypes.byref(desc), _code(dtype), buf, 96)
    if path < 0:
        raise L.SelError(f"sel_dconv_kernel: invalid descriptor: {L.load().sel_last_error().decode()}")
    return PATH_NAMES[path], buf.value.decode()


def _meta(d, x, out, tag):
    """(kernel name, algorithmic bytes, flops) of one launch for the bench
    timer: launches are classified by the kernel they run (the name rocprofv3
    lists), so the live roofline and the kernel trace group the same launches."""
    es = x.element_size()
    width = d.So * d.Ng
    flops = 2.0 * d.B * d.Tvalid * d.G * width * d.K * d.S * d.Cg
    nbytes = es * (d.B * d.Tvs * d.ldx + d.B * d.Tvo * d.ldo + d.G * width * d.K * d.S * d.Cg)
    return (kernel(d, x.dtype)[1], nbytes, flops)


class _DwgradJob(ctypes.Structure):
    """sel_dwgrad_job (include/sel.h)."""
    _fields_ = [(n, ctypes.c_void_p) for n in ("part", "bpart", "v", "wg", "gw", "gg", "gb")] + \
               [(n, ctypes.c_int32) for n in ("N", "Cg", "Kt", "stride", "pad", "G", "nsplit", "bsplit")]


# SEL_DWGRAD_MERGE=0: one final-reduction launch per layer (sel_dconv_wgrad)
# instead of one per sub-discriminator chain (sel_dconv_wgrad_finish_many)
DWGRAD_MERGE = os.environ.get("SEL_DWGRAD_MERGE", "1") != "0"


def wgrad(sp, desc, gout, x, w_or_v, wg, want_w, want_b, pending=None):
    """(gw or gv, gg, gb) of one layer (fp32, torch layouts).  With a `pending`
    list the final reduction is left to finish_pending(pending): the tensors
    are written when it has run (stream order)."""
    lib = L.lib()
    ws = L.workspace(lib.sel_dconv_wgrad_workspace(ctypes.byref(desc), _code(x.dtype)), x.device)
    gw = torch.empty(w_or_v.shape, dtype=torch.float32, device=x.device)
    gg = torch.empty(wg.shape, dtype=torch.float32, device=x.device) if wg is not None else None
    gb = torch.empty(sp.cout, dtype=torch.float32, device=x.device) if want_b else None
    v = w_or_v.detach().contiguous().float() if wg is not None else None
    g = wg.detach().contiguous().float() if wg is not None else None
    args = (ctypes.byref(desc), _code(x.dtype), L.ptr(gout), L.ptr(x), sp.cout, sp.cin // sp.groups, sp.Kt, sp.stride,
            sp.pad, L.ptr(v), L.ptr(g), L.ptr(gw), L.ptr(gg), L.ptr(gb), L.ptr(ws), ws.numel())
    if pending is None:
        L.call("sel_dconv_wgrad", *args, L.stream())
    else:
        job = _DwgradJob()
        L.call("sel_dconv_wgrad_partials", *args, ctypes.byref(job), L.stream(),
               meta=lambda: _wgrad_meta(desc, x, gout))
        pending.append((job, ws, v, g))  # the finish reads ws, v and g
    return (gw if want_w else None), gg, gb


def _wgrad_meta(d, x, gout):
    """(tag, algorithmic bytes, flops) of one weight-gradient partial launch:
    the forward's contraction over the same operands (read x and gout once)."""
    width = d.So * d.Ng
    flops = 2.0 * d.B * d.Tvalid * d.G * width * d.K * d.S * d.Cg
    nbytes = x.numel() * x.element_size() + gout.numel() * gout.element_size()
    return f"dconv_wgrad_partials[G={d.G},Cg={d.Cg},K={d.K},S={d.S},T={d.Tvalid}]", nbytes, flops


def finish_pending(pending):
    """The final weight-gradient reductions of the layers in `pending`, one launch."""
    if pending:
        jobs = (_DwgradJob * len(pending))(*[p[0] for p in pending])
        L.call("sel_dconv_wgrad_finish_many", ctypes.cast(jobs, ctypes.c_void_p), len(pending), L.stream())
        pending.clear()


def _cast(x, dtype):
    from .convops import _cast_raw
    return x if x.dtype == dtype else _cast_raw(x.contiguous(), dtype)


def _view(y, kind, B, T, p):
    """Reference-layout view of a layer buffer (no copy)."""
    if kind == "scale":  # (B, T_alloc, C) -> (B, C, T)
        return y[:, :T, :].permute(0, 2, 1)
    # period: (B*p, L_alloc, C) -> (B, C, L, p)
    Bp, La, C = y.shape
    return y.view(B, p, La, C)[:, :, :T, :].permute(0, 3, 2, 1)


def chain_forward(x0, T0, specs, slope, wn, params, lo=0, hi=None, bufs=None):
    """The layers of one sub-discriminator over the sequences [lo, hi) of x0
    (Bs, T0_alloc, 1) into the per-layer buffers `bufs` (allocated for all Bs
    sequences when None; other sequences are left as they are).  Returns
    (bufs, geo).  Each output row runs the same kernels whatever the launch's
    sequence count; the flat tiling may put a sequence in another tile, so a
    chain run in two halves is held to the concatenated run at 1e-6 (fp32) /
    1e-3 (bf16) norm-wise by tests/test_gpu_gan.py, not to bit equality."""
    dtype = x0.dtype
    Bs = x0.shape[0]
    hi = Bs if hi is None else hi
    geo = chain_layout(specs, T0, x0.shape[1])
    if bufs is None:
        bufs = [torch.empty(Bs, g[3], sp.cout, dtype=dtype, device=x0.device) for sp, g in zip(specs, geo)]
    x = x0
    for li, (sp, g) in enumerate(zip(specs, geo)):
        w, wg, b = _layer_params(params, li, wn)
        T_in, T_alloc_in, T_out, T_out_alloc = g
        d = _fwd_desc(sp, hi - lo, T_in, T_alloc_in, T_out, T_out_alloc, slope)
        y = bufs[li]
        prim(d, x[lo:hi], pack(sp, w, wg, dtype, 0), y[lo:hi],
             bias=b.detach().float().contiguous() if b is not None else None, tag=f"_fwd{li}")
        x = y
    return bufs, geo


class ChainFn(torch.autograd.Function):
    """One sub-discriminator: x0 (Bs, T0_alloc, 1) in the compute dtype with T0
    valid rows -> the reference-layout views of every layer's output.

    forward(ctx, x0, T0, specs, slope, wn, kind, B, p, frozen, pre, *params):
    params per layer are (w, bias) or, with weight norm (wn), (weight_v,
    weight_g, bias); frozen = the parameters are constants here (no
    weight-gradient kernels, no gradient returned for them); pre = None, or
    (lo, bufs): the sequences below lo are already in bufs (chain_forward run
    earlier with the same weights) and only [lo, Bs) is computed — the backward
    still covers all Bs sequences."""

    @staticmethod
    def forward(ctx, x0, T0, specs, slope, wn, kind, B, p, frozen, pre, *params):
        L.need_device(x0)
        ctx.set_materialize_grads(False)  # unused feature maps arrive as None
        dtype = x0.dtype
        per = 3 if wn else 2
        # every stale packed form of the chain in one launch (forward forms, and
        # the adjoint forms when a gradient can flow back through the chain)
        adj = any(ctx.needs_input_grad)
        items = []
        for li, sp in enumerate(specs):
            w, wg, _b = _layer_params(params, li, wn)
            items += [(sp, w, wg, dtype, m) for m in ((0, 1) if adj else (0,))]
        DPACKS.prefetch(items)
        lo, pb = pre if pre is not None else (0, None)
        bufs, geo = chain_forward(x0, T0, specs, slope, wn, params, lo, None, pb)
        views = [_view(y, kind, B, g[2], p) for y, g in zip(bufs, geo)]
        ctx.save_for_backward(x0, *bufs, *params)
        ctx.cfg = (specs, slope, wn, geo, len(bufs), kind, B, p, per, frozen)
        return tuple(views)

    @staticmethod
    def backward(ctx, *gviews):
        saved = ctx.saved_tensors
        specs, slope, wn, geo, nl, kind, B, p, per, frozen = ctx.cfg
        x0, bufs, params = saved[0], saved[1:1 + nl], saved[1 + nl:]
        dtype = x0.dtype
        Bs = x0.shape[0]
        npre = 10  # leading non-param inputs of forward
        pgrads = [None] * len(params)

        def ext(li):
            g = gviews[li]
            return None if g is None else _as_buffer(g, bufs[li], kind, B, geo[li][2], p)

        top = max((li for li in range(nl) if gviews[li] is not None), default=None)
        if top is None:
            return (None,) * (npre + len(params))
        pending = [] if DWGRAD_MERGE else None  # the chain's final reductions: one launch at the end
        g = ext(top)
        gpre = _lrelu_bwd(g, bufs[top], slope) if specs[top].leaky else g
        gx0 = None
        for li in range(top, -1, -1):
            sp = specs[li]
            T_in, T_alloc_in, T_out, T_out_alloc = geo[li]
            w, wg, b = _layer_params(params, li, wn)
            x_in = bufs[li - 1] if li > 0 else x0
            base = npre + per * li
            need_w = ctx.needs_input_grad[base] and not frozen
            need_g = wn and ctx.needs_input_grad[base + 1] and not frozen
            need_b = b is not None and ctx.needs_input_grad[base + per - 1] and not frozen
            if need_w or need_g or need_b:
                d_f = _fwd_desc(sp, Bs, T_in, T_alloc_in, T_out, T_out_alloc, slope)
                gw, gg, gb = wgrad(sp, d_f, gpre, x_in, w, wg, True, need_b, pending)
                pgrads[per * li] = gw if need_w else None
                if wn:
                    pgrads[per * li + 1] = gg if need_g else None
                if need_b:
                    pgrads[per * li + per - 1] = gb
            if li == 0 and not ctx.needs_input_grad[0]:
                break
            # adjoint of this layer: the previous layer's feature-map gradient is
            # added and its LeakyReLU' applied in the same epilogue
            d_b = _dgrad_desc(sp, Bs, T_alloc_in, T_out, T_out_alloc, slope, li > 0, T_in=T_in)
            wd = pack(sp, w, wg, dtype, 1)
            gin = torch.empty(Bs, T_alloc_in, sp.cin, dtype=dtype, device=x0.device)
            res = aux = None
            if li > 0:
                res = ext(li - 1)
                if not specs[li - 1].leaky:
                    raise NotImplementedError("inner discriminator layers are LeakyReLU layers")
                aux = bufs[li - 1]
            prim(d_b, gpre, wd, gin, aux=aux, res=res, tag=f"_dgrad{li}")
            if li == 0:
                gx0 = gin
            gpre = gin
        finish_pending(pending)
        return (gx0, None, None, None, None, None, None, None, None, None, *pgrads)


def _layer_params(params, li, wn):
    if wn:
        return params[3 * li], params[3 * li + 1], params[3 * li + 2]
    return params[2 * li], None, params[2 * li + 1]


def _lrelu_bwd(g, y, slope):
    """g * LeakyReLU'(y) (the top layer's external gradient; elementwise)."""
    return torch.where(y > 0, g, g * slope)


def _as_buffer(g, y, kind, B, T, p):
    """Gradient of a feature-map view -> y's (Bs, T_alloc, C) buffer layout
    (rows past the valid length are never read).  A gradient written by the GAN
    loss kernels into a same-strided buffer is used in place."""
    v = _view(y, kind, B, T, p)
    if (g.dtype == y.dtype and tuple(g.stride()) == tuple(v.stride()) and g.storage_offset() == 0
            and g.untyped_storage().nbytes() >= y.numel() * y.element_size()):
        return torch.as_strided(g, y.shape, y.stride(), 0)
    buf = torch.empty_like(y)
    _view(buf, kind, B, T, p).copy_(g)
    return buf


# ---------------------------------------------------------------------------
# front-ends: MSD average pooling, MPD reflect-pad + period fold
# ---------------------------------------------------------------------------
class AvgPoolFn(torch.autograd.Function):
    """AvgPool1d(kernel, stride, padding) over (B, T) fp32 rows (count_include_pad)."""

    @staticmethod
    def forward(ctx, x, kernel, stride, pad):
        L.need_device(x)
        B, T = x.shape
        To = (T + 2 * pad - kernel) // stride + 1
        y = torch.empty(B, To, dtype=torch.float32, device=x.device)
        xc = x.contiguous()
        L.call("sel_avgpool1d_fwd", L.ptr(xc), B, T, T, kernel, stride, pad, To, To, L.ptr(y), L.stream())
        ctx.cfg = (B, T, kernel, stride, pad, To)
        return y

    @staticmethod
    def backward(ctx, gy):
        B, T, kernel, stride, pad, To = ctx.cfg
        gy = gy.contiguous()
        gx = torch.empty(B, T, dtype=torch.float32, device=gy.device)
        L.call("sel_avgpool1d_bwd", L.ptr(gy), B, T, T, kernel, stride, pad, To, To, L.ptr(gx), L.stream())
        return gx, None, None, None


class MpdFoldFn(torch.autograd.Function):
    """(B, T) fp32 -> (B*p, L_alloc) sequences of the period grid (reflect pad)."""

    @staticmethod
    def forward(ctx, x, p, Lalloc):
        L.need_device(x)
        B, T = x.shape
        y = torch.empty(B * p, Lalloc, dtype=torch.float32, device=x.device)
        xc = x.contiguous()
        L.call("sel_mpd_fold", L.ptr(xc), B, T, T, p, Lalloc, L.ptr(y), L.stream())
        ctx.cfg = (B, T, p, Lalloc)
        return y

    @staticmethod
    def backward(ctx, gy):
        B, T, p, Lalloc = ctx.cfg
        gy = gy.contiguous()
        gx = torch.empty(B, T, dtype=torch.float32, device=gy.device)
        L.call("sel_mpd_unfold", L.ptr(gy), B, T, T, p, Lalloc, L.ptr(gx), L.stream())
        return gx, None, None


# ---------------------------------------------------------------------------
# GAN losses (losses/adversarial_loss.py, losses/feat_match_loss.py)
# ---------------------------------------------------------------------------
L1, MSE, HINGE_REAL, HINGE_FAKE, SUM = 0, 1, 2, 3, 4


def _view_args(t):
    nd = t.dim()
    size = (ctypes.c_int64 * nd)(*t.shape)
    stride = (ctypes.c_int64 * nd)(*t.stride())
    return size, stride, nd


def _memory_order(t):
    """Dim permutation that walks `t` in memory order (largest stride outermost):
    the kernels iterate the LAST dim fastest, so a (B, C, T) view of a
    channels-last buffer is read row by row, coalesced."""
    return sorted(range(t.dim()), key=lambda d: (-t.stride(d), -t.shape[d]))


class GanReduceFn(torch.autograd.Function):
    """scale * sum over elements of a (strided view) of |a - b| (kind L1),
    (a - target)^2 (MSE) or the hinge terms; gradient w.r.t. a only (b is the
    detached real-data feature map, feat_match_loss.py:47)."""

    @staticmethod
    def forward(ctx, a, b, kind, target, scale):
        L.need_device(a)
        if a.dim() > 4:
            raise ValueError("GAN loss views have at most 4 dims")
        perm = _memory_order(a)
        sa, ta, nd = _view_args(a.permute(perm))
        if b is not None:
            if b.shape != a.shape or b.dtype != a.dtype:
                raise ValueError(f"feature maps differ: {tuple(a.shape)}/{a.dtype} vs {tuple(b.shape)}/{b.dtype}")
            sb, tb, _ = _view_args(b.permute(perm))
        else:
            sb = tb = None
        out = torch.empty((), dtype=torch.float32, device=a.device)
        ws = L.workspace(L.lib().sel_gan_workspace(), a.device)
        L.call("sel_gan_reduce", kind, _code(a.dtype), L.ptr(a), sa, ta, L.ptr(b), sb, tb, nd, float(target),
               float(scale), 0, L.ptr(out), L.ptr(ws), ws.numel(), L.stream())
        ctx.save_for_backward(a, b)
        ctx.cfg = (kind, target, scale)
        return out

    @staticmethod
    def backward(ctx, g):
        a, b = ctx.saved_tensors
        kind, target, scale = ctx.cfg
        perm = _memory_order(a)
        sa, ta, nd = _view_args(a.permute(perm))
        sb, tb = (None, None) if b is None else _view_args(b.permute(perm))[:2]
        # same strides as the view, over a full copy of its base storage, so the
        # discriminator backward can consume it in place (sel.dconvops._as_buffer)
        base = a._base if a._base is not None else a
        gbuf = torch.empty_like(base) if base is not a else torch.empty_like(a)
        ga = torch.as_strided(gbuf, a.shape, a.stride(), a.storage_offset()) if base is not a else gbuf
        gs = (ctypes.c_int64 * nd)(*ga.permute(perm).stride())
        # the upstream scalar is read in place (the kernel multiplies by `scale`):
        # no separate scaling launch per term
        gc = g if (g.dtype == torch.float32 and g.numel() == 1) else g.float().reshape(1).contiguous()
        L.call("sel_gan_grad", kind, _code(a.dtype), L.ptr(a), sa, ta, L.ptr(b), sb, tb, nd, float(target),
               ctypes.c_void_p(gc.data_ptr()), float(scale), L.ptr(ga), gs, 0, L.stream())
        return ga, None, None, None, None


def l1_mean(a, b, weight=1.0):
    """weight * mean |a - b| (the weight folded into the kernel's scale)."""
    return GanReduceFn.apply(a, b.detach(), L1, 0.0, float(weight) / a.numel())


def mse_to(a, target):
    return GanReduceFn.apply(a, None, MSE, float(target), 1.0 / a.numel())


def hinge(a, real):
    return GanReduceFn.apply(a, None, HINGE_REAL if real else HINGE_FAKE, 0.0, -1.0 / a.numel())


def neg_mean(a):
    return GanReduceFn.apply(a, None, SUM, 0.0, -1.0 / a.numel())
