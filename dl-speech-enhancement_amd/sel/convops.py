"""Autograd ops over the conv-stack kernels of libsel.so.

Activations live channels-last in HBM: a (B, C, T) tensor handed between the
drop-in modules is a transposed *view* of a contiguous (B, T, C) buffer, so the
reference's (B, C, T) module API is kept with zero layout copies.

Reference semantics (file:line under the reference root):
* CausalConv1d            layers/conv_layer.py:109-150 (left zero pad (k-1)*d)
* CausalConvTranspose1d   layers/conv_layer.py:153-191 (replicate pad 1, crop [s:-s])
* Conv1d1x1               layers/conv_layer.py:19-23
* CausalResidualUnit      models/autoencoder/modules/residual_unit.py:43-80
"""
import ctypes
import os
import threading
import weakref
from contextlib import contextmanager

import torch
from torch.optim.optimizer import register_optimizer_step_post_hook as _register_optimizer_step_post_hook

from . import _lib as L

F32, BF16 = 0, 1
PAD_ZERO, PAD_REPLICATE = 0, 1
PACK_FWD, PACK_FWD_STRIDED, PACK_CONVT = 0, 1, 2


class ConvDesc(ctypes.Structure):
    _fields_ = [("rows", ctypes.c_int64), ("T", ctypes.c_int32), ("C", ctypes.c_int32),
                ("N", ctypes.c_int32), ("K", ctypes.c_int32), ("dil", ctypes.c_int32),
                ("pad", ctypes.c_int32), ("pad_mode", ctypes.c_int32), ("in_elu", ctypes.c_int32),
                ("bias_period", ctypes.c_int32)]

    def adjoint(self):
        """dgrad of this primitive: same primitive on gout with Wd[C][K][N]."""
        return ConvDesc(self.rows, self.T, self.N, self.C, self.K, self.dil,
                        (self.K - 1) * self.dil - self.pad, PAD_ZERO, 0, 0)

    def with_(self, **kw):
        d = ConvDesc(*[getattr(self, f) for f, _ in self._fields_])
        for k, v in kw.items():
            setattr(d, k, v)
        return d


_state = threading.local()


def compute_dtype():
    return getattr(_state, "dtype", torch.float32)


@contextmanager
def precision(dtype):
    """Run the conv stack in `dtype` (torch.float32 = parity path, torch.bfloat16 =
    bf16 MFMA with fp32 accumulation).  Parameters and their grads stay fp32."""
    prev = compute_dtype()
    _state.dtype = dtype
    try:
        yield
    finally:
        _state.dtype = prev


def _code(dtype):
    if dtype == torch.float32:
        return F32
    if dtype == torch.bfloat16:
        return BF16
    raise TypeError(f"unsupported activation dtype {dtype}")


def to_cl(x):
    """(B, C, T) tensor -> contiguous (B, T, C) storage (a view when possible)."""
    y = x.transpose(1, 2)
    return y if y.is_contiguous() else y.contiguous()


def _cast_raw(x, dtype):
    out = torch.empty(x.shape, dtype=dtype, device=x.device)
    xc = x.contiguous()
    L.call("sel_cast", L.ptr(xc), _code(xc.dtype), L.ptr(out), _code(dtype), xc.numel(), L.stream())
    return out


class _CastFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, dtype):
        ctx.src = x.dtype
        return _cast_raw(x, dtype)

    @staticmethod
    def backward(ctx, g):
        return _cast_raw(g, ctx.src), None


def cast(x, dtype):
    """dtype cast on device (sel_cast), differentiable."""
    if x.dtype == dtype:
        return x
    L.need_device(x)
    if torch.is_grad_enabled() and x.requires_grad:
        return _CastFn.apply(x, dtype)
    return _cast_raw(x, dtype)


def pack(kind, w, stride, dtype):
    """fp32 torch weight -> packed (dtype) Wp[N][K][C] on device."""
    if kind == PACK_CONVT:
        cin, cout, k = w.shape
        shape = (stride * cout, 2, cin)
    else:
        cout, cin, k = w.shape
        shape = (cout, k, cin) if kind == PACK_FWD else (cout, 3, stride * cin)
    wc = w.detach().contiguous().float()
    out = torch.empty(shape, dtype=dtype, device=w.device)
    L.call("sel_pack_weight", kind, L.ptr(wc), cout, cin, k, stride, _code(dtype), L.ptr(out), L.stream())
    return out


def pack_dgrad(wp):
    N, K, C = wp.shape
    out = torch.empty((C, K, N), dtype=wp.dtype, device=wp.device)
    L.call("sel_pack_dgrad", L.ptr(wp), N, K, C, _code(wp.dtype), L.ptr(out), L.stream())
    return out


class _PackJob(ctypes.Structure):
    """include/sel.h sel_pack_job"""
    _fields_ = [("w", ctypes.c_void_p), ("wpack", ctypes.c_void_p), ("wdgrad", ctypes.c_void_p),
                ("offset", ctypes.c_int64), ("kind", ctypes.c_int32), ("cout", ctypes.c_int32),
                ("cin", ctypes.c_int32), ("k", ctypes.c_int32), ("stride", ctypes.c_int32),
                ("reserved", ctypes.c_int32)]


def _packed_shape(kind, w, stride):
    if kind == PACK_CONVT:
        cin, cout, k = w.shape
        return (stride * cout, 2, cin), cout, cin, k
    cout, cin, k = w.shape
    return ((cout, k, cin) if kind == PACK_FWD else (cout, 3, stride * cin)), cout, cin, k


class _PackEntry:
    __slots__ = ("wref", "pid", "kind", "stride", "dtype", "version", "wp", "wd")


class PackCache:
    """Packed bf16/fp32 forms (fwd Wp and dgrad Wd) of every conv weight, refreshed
    in ONE sel_pack_many launch per weight update instead of two launches per
    layer per step.

    Two staleness signals, because neither alone is complete:
    * the parameter's version counter, bumped by in-place updates through
      autograd-visible ops (copy_, load_state_dict, foreach/for-loop Adam);
    * a global optimizer step post-hook (``_optimizer_stepped``), because
      torch's fused Adam (``fused=True``, the GPU default here) writes the
      parameters in a kernel that does NOT bump ``_version`` — with the version
      alone every later forward would silently reuse the step-0 packs.
    A refresh repacks every stale entry into FRESH buffers, so tensors saved by
    a graph that has not run backward yet are never overwritten.  Code that
    mutates a weight through ``.data`` (which has its own version counter) must
    call ``invalidate()``.
    """

    def __init__(self):
        self._entries = {}
        self._by_param = {}  # id(param) -> [entry keys]
        self._lock = threading.Lock()

    def invalidate(self):
        with self._lock:
            self._entries.clear()
            self._by_param.clear()

    def mark_stale(self, params):
        """Force a repack of every entry packed from one of `params`."""
        with self._lock:
            for p in params:
                for key in self._by_param.get(id(p), ()):
                    e = self._entries.get(key)
                    if e is not None and e.wref() is p:
                        e.version = None

    def get(self, kind, w, stride, dtype):
        key = (w.data_ptr(), kind, stride, dtype, tuple(w.shape), w.device)
        with self._lock:
            e = self._entries.get(key)
            if e is not None and e.wref() is w and e.version == w._version:
                return e.wp, e.wd
            if e is None or e.wref() is not w:
                e = _PackEntry()
                e.wref, e.pid, e.kind, e.stride, e.dtype = weakref.ref(w), id(w), kind, stride, dtype
                e.version, e.wp, e.wd = None, None, None
                self._entries[key] = e
                keys = self._by_param.setdefault(id(w), [])
                if key not in keys:
                    keys.append(key)
            self._refresh(w.device, dtype)
            return e.wp, e.wd

    def _refresh(self, device, dtype):
        stale = []
        for key, e in list(self._entries.items()):
            w = e.wref()
            if w is None:
                del self._entries[key]
                keys = self._by_param.get(e.pid)
                if keys is not None and key in keys:
                    keys.remove(key)
                    if not keys:
                        del self._by_param[e.pid]
                continue
            if e.dtype == dtype and w.device == device and e.version != w._version:
                stale.append((e, w))
        if not stale:
            return
        shapes = []
        total = 0
        for e, w in stale:
            shp, cout, cin, k = _packed_shape(e.kind, w, e.stride)
            n = shp[0] * shp[1] * shp[2]
            if n >= 1 << 31 or w.numel() >= 1 << 31:
                raise L.SelError("sel: a packed conv weight must stay below 2^31 elements")
            shapes.append((shp, cout, cin, k, total, n))
            total += n
        flat = torch.empty(2 * total, dtype=dtype, device=device)
        jobs = (_PackJob * len(stale))()
        for j, ((e, w), (shp, cout, cin, k, off, n)) in enumerate(zip(stale, shapes)):
            if not w.is_contiguous() or w.dtype != torch.float32:
                raise L.SelError("sel: conv weights must be contiguous fp32 parameters")
            e.wp = flat[off:off + n].view(shp)
            e.wd = flat[total + off:total + off + n].view(shp[2], shp[1], shp[0])
            e.version = w._version
            jobs[j] = _PackJob(w.data_ptr(), e.wp.data_ptr(), e.wd.data_ptr(), off, e.kind, cout, cin, k,
                               e.stride, 0)
        # the job table goes in the kernel arguments (no pinned staging, no
        # host-to-device copy: that pair left the GPU idle ~0.3 ms per C3 step);
        # SEL_PACK_HOST=0: the device-table form (A/B)
        if PACK_HOST:
            L.call("sel_pack_many_host", ctypes.cast(jobs, ctypes.c_void_p), len(stale), total, _code(dtype),
                   L.stream())
        else:
            host = torch.frombuffer(bytearray(jobs), dtype=torch.uint8).pin_memory()
            dev = host.to(device, non_blocking=True)
            L.call("sel_pack_many", L.ptr(dev), len(stale), total, _code(dtype), L.stream())


PACK_HOST = os.environ.get("SEL_PACK_HOST", "1") != "0"
PACKS = PackCache()


def _optimizer_stepped(optimizer, args, kwargs):
    """Global torch.optim post-step hook: every conv weight the optimizer
    updated is repacked before its next use (see PackCache: fused Adam does not
    bump the parameters' version counters).  torch's optimizers skip parameters
    whose .grad is None (the frozen decoder and quantizer of the denoise
    trainer), so those keep their packs."""
    PACKS.mark_stale(p for g in optimizer.param_groups for p in g["params"] if p.grad is not None)


_register_optimizer_step_post_hook(_optimizer_stepped)


def prim(desc, x, wp, bias=None, aux=None, res=None, out_dtype=None):
    """The conv primitive; x is (rows, C) channels-last (any leading shape)."""
    out_dtype = out_dtype or x.dtype
    out = torch.empty((desc.rows, desc.N), dtype=out_dtype, device=x.device)
    for t in (aux, res):
        if t is not None:
            assert t.dtype == out_dtype and t.is_contiguous() and t.numel() == out.numel()
    assert x.is_contiguous() and x.numel() == desc.rows * desc.C and wp.dtype == x.dtype
    L.call("sel_conv_fwd", ctypes.byref(desc), _code(x.dtype), _code(out_dtype), L.ptr(x), L.ptr(wp),
           L.ptr(bias), L.ptr(aux), L.ptr(res), L.ptr(out), L.stream(),
           meta=lambda: _fwd_meta(desc, x, out, wp, aux, res))
    return out


def fwd_kernel_name(desc, in_dtype, out_dtype, has_epilogue=False):
    """rocprof name fragment of the kernel instance a launch uses."""
    kid = L.lib().sel_conv_fwd_kernel_id(ctypes.byref(desc), _code(in_dtype), _code(out_dtype), int(has_epilogue))
    if kid < 0:
        return f"k_conv_fwd<{in_dtype}>"
    if kid >= 10 ** 9:  # weight-stationary thin kernel: 1e9 + E*5e8 + ((R/32*1000 + C)*1000 + N)*10 + K
        kid -= 10 ** 9
        e, kid = kid >= 5 * 10 ** 8, kid % (5 * 10 ** 8)
        k, n, c, r = kid % 10, (kid // 10) % 1000, (kid // 10000) % 1000, 32 * (kid // 10000000)
        return f"k_conv_thin_bf16<{c}, {n}, {k}, {r}, {'true' if e else 'false'}>"
    to = "bf16" if out_dtype == torch.bfloat16 else "float"
    if kid >= 94 * 10 ** 7:  # sample-tile warp-specialised kernel (conv_wss.hip): 9.4e8 + 1e6 (SPT-1) + 1e4 BN + 10 S + K
        r = kid - 94 * 10 ** 7
        spt, r = r // 10 ** 6 + 1, r % 10 ** 6
        return f"k_conv_wss<{r % 10}, {(r // 10) % 1000}, {r // 10000}, {to}" + (f", {spt}>" if spt > 1 else ">")
    if kid >= 93 * 10 ** 7:  # pointwise (1x1) weight-stationary kernel: 9.3e8 + N
        n = kid - 93 * 10 ** 7
        return f"k_pw_bf16<{n}, {n}"
    if kid >= 92 * 10 ** 7:  # eight-wave warp-specialised kernel, 256 x 128 tiles of 64 x 64 wave tiles: 9.2e8 + K
        return f"k_conv_ws8<{kid - 92 * 10 ** 7}, {to}, 256, 128, 64, 2>"
    if kid >= 91 * 10 ** 7:  # eight-wave warp-specialised kernel, 512 x 128 tiles: 9.1e8 + K
        return f"k_conv_ws8<{kid - 91 * 10 ** 7}, {to}, 512, 128>"
    if kid >= 9 * 10 ** 8:  # warp-specialised kernel (12 waves): 9e8 + K
        return f"k_conv_ws_bf16<{kid - 9 * 10 ** 8}, {to}>"
    kmax, kid = kid % 10, kid // 10
    wm, kid = kid % 10, kid // 10
    bm, bn = kid // 1000, kid % 1000
    return f"k_conv_fwd_bf16<{bm}, {bn}, {wm}, {kmax}, {to}>"


def _fwd_meta(desc, x, out, wp, aux, res):
    """(kernel tag, algorithmic HBM bytes, flops) of one primitive launch:
    read the input rows once, the packed weights once, aux/res once, write out once."""
    es = x.element_size()
    nbytes = desc.rows * desc.C * es + out.numel() * out.element_size() + wp.numel() * es
    for t in (aux, res):
        if t is not None:
            nbytes += t.numel() * t.element_size()
    flops = 2.0 * desc.rows * desc.N * desc.K * desc.C
    return fwd_kernel_name(desc, x.dtype, out.dtype, aux is not None or res is not None), nbytes, flops


def wgrad(desc, gout, x, want_bias):
    lib = L.lib()
    ws = L.workspace(lib.sel_conv_wgrad_workspace(ctypes.byref(desc)), x.device)
    gwp = torch.empty((desc.N, desc.K, desc.C), dtype=torch.float32, device=x.device)
    gb = torch.empty(desc.bias_period, dtype=torch.float32, device=x.device) if want_bias else None
    L.call("sel_conv_wgrad", ctypes.byref(desc), _code(x.dtype), L.ptr(gout), L.ptr(x), L.ptr(gwp),
           L.ptr(gb), L.ptr(ws), ws.numel(), L.stream())
    return gwp, gb


class _WgradJob(ctypes.Structure):
    """include/sel.h sel_wgrad_job"""
    _fields_ = [("part", ctypes.c_void_p), ("gw", ctypes.c_void_p), ("gb", ctypes.c_void_p),
                ("nw", ctypes.c_int64), ("nsplit", ctypes.c_int32), ("N", ctypes.c_int32),
                ("bias_period", ctypes.c_int32), ("kind", ctypes.c_int32), ("cout", ctypes.c_int32),
                ("cin", ctypes.c_int32), ("k", ctypes.c_int32), ("stride", ctypes.c_int32)]


# Deferred weight-gradient reductions (SEL_WGRAD_DEFER=0: off).  Inside a
# backward pass every layer's split-row partial kernel runs where the layer's
# gradient is produced, but the reductions of all layers run as ONE launch
# (sel_wgrad_finish_many) from an autograd final callback, i.e. before
# backward() returns and before anything reads a .grad: ~25 reduction launches
# of 5-10 us per C3 step become one.  Only where nothing can read the gradient
# tensor in between: the parameter is a leaf whose .grad is None (AccumulateGrad
# then takes the returned tensor itself, no copy or add) and has no tensor or
# post-accumulate hook (a hook that reads .grad early should set
# SEL_WGRAD_DEFER=0 if it is attached some other way), no create_graph.  Under
# a multi-rank process group a layer defers only when every parameter it feeds
# belongs to a sel.ddp.GradBuckets reducer: the returned gradient is then a
# view of the parameter's slot in the reducer's flat buffer, and the reducer
# runs the pending reductions of a bucket (flush_params) when the bucket's last
# gradient has arrived, right before its all-reduce.  The flush checks that
# every deferred tensor is still the one AccumulateGrad kept and raises
# otherwise.
WGRAD_DEFER = os.environ.get("SEL_WGRAD_DEFER", "1") != "0"
_DEFERRED = []
_DEFER_LOCK = threading.Lock()
# Deferred partial kernels on a side stream (SEL_WGRAD_STREAM=1): a layer's
# weight-gradient partials depend only on its gout and input, which the
# backward's next dgrad launches do not change, so they can run beside that
# chain and fill the CUs its launches leave idle; the batched reduction runs
# on the side stream and the current stream waits for it before backward()
# returns.  Same kernels, same bits.
WGRAD_STREAM = os.environ.get("SEL_WGRAD_STREAM", "0") != "0"
_WG_STREAMS = {}


def _wgrad_stream(device):
    s = _WG_STREAMS.get(device.index)
    if s is None:
        s = _WG_STREAMS[device.index] = torch.cuda.Stream(device=device)
    return s


def _can_defer(params):
    """params: the leaf parameters the returned gradients go to, in order (gw, gb)."""
    if not WGRAD_DEFER or torch.is_grad_enabled() or not params:
        return False
    try:
        import torch.distributed as dist
        # data parallel: only parameters of a sel.ddp reducer, which runs the
        # pending reductions of a bucket before its all-reduce, may wait
        owned = all(p is not None and _owner(p) is not None for p in params)
        if owned and not DDP_DEFER:
            return False
        # (any process group: torch's DDP may wrap the module even at one rank)
        if not owned and dist.is_available() and dist.is_initialized():
            return False
        for p in params:
            if p is None or not p.is_leaf or p.grad is not None:
                return False
            # a tensor hook or a post-accumulate hook (e.g. an optimizer-in-backward)
            # would read the gradient before the final callback computes it (the
            # reducer's own arrival hook reads no values)
            if getattr(p, "_backward_hooks", None) or (getattr(p, "_post_accumulate_grad_hooks", None)
                                                       and not owned):
                return False
            # the engine accumulates into .grad in this backward (not autograd.grad(inputs=...))
            if not torch._C._will_engine_execute_node(torch.autograd.graph.get_gradient_edge(p).node):
                return False
    except (ImportError, RuntimeError, AttributeError):
        return False
    return True


def _queue_flush():
    """Arrange the batched reduction at the end of the running backward pass
    (False outside one: then nothing may be deferred)."""
    try:
        torch.autograd.Variable._execution_engine.queue_callback(_flush_deferred)
    except RuntimeError:  # not inside a backward pass
        return False
    return True


def _defer(job, ws, params, gw, gb, st):
    refs = [(weakref.ref(params[0]), gw.data_ptr())] + \
        ([(weakref.ref(params[1]), gb.data_ptr())] if gb is not None else [])
    # (no reference to gw / gb here: AccumulateGrad takes the returned tensor
    # itself as .grad only while nothing else holds it)
    with _DEFER_LOCK:
        _DEFERRED.append((job, ws, refs, st.value))


# ---------------------------------------------------------------------------
# data parallel: the deferred reductions run per gradient bucket (sel.ddp)
# ---------------------------------------------------------------------------
DDP_DEFER = os.environ.get("SEL_DDP_DEFER", "1") != "0"
_REDUCERS = []     # weakrefs to sel.ddp.GradBuckets
DDP_STATS = {"bucket_flushes": 0, "jobs": 0}


def register_grad_buckets(reducer):
    """A module wrapped again: the older reducer of any of its parameters is
    detached (hooks removed, dropped from the registry), so exactly one reducer
    owns a parameter; dead references are pruned."""
    live = []
    for ref in _REDUCERS:
        r = ref()
        if r is None:
            continue
        if any(s[3]() is not None and reducer.owns(s[3]()) for s in list(r.slots.values())):
            r.detach()
            continue
        live.append(ref)
    live.append(weakref.ref(reducer))
    _REDUCERS[:] = live


def _owner(p):
    for ref in _REDUCERS:
        r = ref()
        if r is not None and r.owns(p):
            return r
    return None


def _grad_out(p, shape, device):
    """Gradient tensor of a deferred reduction for parameter p: a view of its
    slot when a data-parallel reducer owns p, else a fresh tensor."""
    r = _owner(p) if p is not None else None
    return r.view(p) if r is not None else torch.empty(shape, dtype=torch.float32, device=device)


def _wgrad_meta(desc, x, nsplit):
    """(tag, algorithmic bytes, flops) of one split-row weight-gradient partial
    launch: read gout and x once, write nsplit fp32 partials of the N x K x C
    weight (the partials are the split design's own traffic, counted)."""
    es = x.element_size()
    nw = desc.N * desc.K * desc.C
    nbytes = desc.rows * (desc.N + desc.C) * es + 4 * nsplit * nw
    return (f"wgrad_partials[N={desc.N},K={desc.K},C={desc.C},T={desc.T}]", nbytes,
            2.0 * desc.rows * desc.N * desc.K * desc.C)


def _finish_meta(group):
    """k_wgrad_finish_many: read every job's fp32 split partials, write its gradient."""
    nbytes = sum(4 * j.nw * (j.nsplit + 1) for j in group)
    return "k_wgrad_finish_many", nbytes, 0.0


def _run_jobs(entries):
    """sel_wgrad_finish_many over deferred entries, one launch per stream."""
    cur = torch.cuda.current_stream()
    for st in dict.fromkeys(e[3] for e in entries):
        group = [e[0] for e in entries if e[3] == st]
        jobs = (_WgradJob * len(group))(*group)
        L.call("sel_wgrad_finish_many", ctypes.cast(jobs, ctypes.c_void_p), len(group), ctypes.c_void_p(st),
               meta=lambda: _finish_meta(group))
        if (st or 0) != cur.cuda_stream:  # (a null-stream handle reads as None)
            # the gradients are read on the current stream from here on (the
            # optimizer / the all-reduce): order it after this finish on ANY
            # other stream, not only the SEL_WGRAD_STREAM side streams
            side = next((s for s in _WG_STREAMS.values() if s.cuda_stream == st), None)
            if side is None:
                side = torch.cuda.ExternalStream(st, device=cur.device)
            cur.wait_stream(side)


def flush_params(params):
    """Run now (one launch) the pending reductions of every layer with a
    parameter in `params` (a data-parallel bucket about to be all-reduced);
    a layer's parameters in other buckets get their values too, before their
    own bucket's all-reduce."""
    ids = {id(p) for p in params}
    with _DEFER_LOCK:
        mine = [e for e in _DEFERRED if any(id(ref()) in ids for ref, _ in e[2] if ref() is not None)]
        if mine:
            keep = {id(e) for e in mine}
            _DEFERRED[:] = [e for e in _DEFERRED if id(e) not in keep]
    if mine:
        _run_jobs(mine)
        DDP_STATS["bucket_flushes"] += 1
        DDP_STATS["jobs"] += len(mine)


def _flush_deferred():
    with _DEFER_LOCK:
        pending = list(_DEFERRED)
        _DEFERRED.clear()
    if not pending:
        return
    for _job, _ws, refs, _st in pending:
        for ref, ptr in refs:
            p_ = ref()
            if p_ is None or p_.grad is None or p_.grad.data_ptr() != ptr:
                raise L.SelError("sel: a deferred weight gradient did not become the parameter's .grad "
                                 "(set SEL_WGRAD_DEFER=0 for this use)")
    # one launch per stream the partial kernels ran on (normally one)
    _run_jobs(pending)
    # the workspaces are released here; the finish kernel is already enqueued on
    # this stream ahead of any later use of that memory


def wgrad_torch(desc, gout, x, kind, w_shape, stride, want_bias, params=None):
    """Weight (torch layout, fp32) and bias gradient of one layer; the unpack is
    fused into the kernel's final reduction pass (sel_conv_wgrad_unpacked).
    `params`: (weight, bias if want_bias) leaf parameters that receive the
    returned gradients (enables the deferred, batched reduction; WGRAD_DEFER)."""
    lib = L.lib()
    ws = L.workspace(lib.sel_conv_wgrad_workspace(ctypes.byref(desc)), x.device)
    if kind == PACK_CONVT:
        cin, cout, k = w_shape
    else:
        cout, cin, k = w_shape
    if params is not None and len(params) == 1 + int(want_bias) and _can_defer(params) and _queue_flush():
        gw = _grad_out(params[0], w_shape, x.device)
        gb = _grad_out(params[1], (desc.bias_period,), x.device) if want_bias else None
        ns = ctypes.c_int()
        st = L.stream()
        if WGRAD_STREAM:
            side = _wgrad_stream(x.device)
            side.wait_stream(torch.cuda.current_stream(x.device))
            for t in (gout, x, ws):
                t.record_stream(side)
            st = ctypes.c_void_p(side.cuda_stream)
        L.call("sel_conv_wgrad_partials", ctypes.byref(desc), _code(x.dtype), L.ptr(gout), L.ptr(x),
               int(want_bias), L.ptr(ws), ws.numel(), ctypes.byref(ns), st,
               meta=lambda: _wgrad_meta(desc, x, ns.value))
        job = _WgradJob(ws.data_ptr(), gw.data_ptr(), gb.data_ptr() if gb is not None else None,
                        desc.N * desc.K * desc.C, ns.value, desc.N, desc.bias_period, kind, cout, cin, k,
                        stride)
        _defer(job, ws, params, gw, gb, st)
        return gw, gb
    gw = torch.empty(w_shape, dtype=torch.float32, device=x.device)
    gb = torch.empty(desc.bias_period, dtype=torch.float32, device=x.device) if want_bias else None
    L.call("sel_conv_wgrad_unpacked", ctypes.byref(desc), _code(x.dtype), L.ptr(gout), L.ptr(x), kind, cout, cin,
           k, stride, L.ptr(gw), L.ptr(gb), L.ptr(ws), ws.numel(), L.stream())
    return gw, gb


def unpack(kind, gwp, w_shape, stride):
    gw = torch.empty(w_shape, dtype=torch.float32, device=gwp.device)
    if kind == PACK_CONVT:
        cin, cout, k = w_shape
    else:
        cout, cin, k = w_shape
    L.call("sel_unpack_wgrad", kind, L.ptr(gwp), cout, cin, k, stride, L.ptr(gw), L.stream())
    return gw


def _layer_desc(kind, B, T_in, cin, cout, k, stride, dil, has_bias):
    """Descriptor + output length for a reference layer in primitive form."""
    if kind == PACK_FWD:
        if stride != 1:
            raise NotImplementedError("stride > 1 conv is lowered through PACK_FWD_STRIDED")
        d = ConvDesc(B * T_in, T_in, cin, cout, k, dil, (k - 1) * dil, PAD_ZERO, 0, cout if has_bias else 0)
        return d, T_in, cout
    if kind == PACK_FWD_STRIDED:
        if T_in % stride:
            raise L.SelError(f"sel: strided conv needs T ({T_in}) divisible by the stride ({stride})")
        To = T_in // stride
        d = ConvDesc(B * To, To, stride * cin, cout, 3, 1, 2, PAD_ZERO, 0, cout if has_bias else 0)
        return d, To, cout
    # transposed: (B, L, Cin) -> (B, L*s, Cout) as (B, L, s*Cout)
    d = ConvDesc(B * T_in, T_in, cin, stride * cout, 2, 1, 1, PAD_REPLICATE, 0, cout if has_bias else 0)
    return d, T_in * stride, cout


def _live(*refs):
    """Parameters behind the weak references of the gradients a wgrad call
    returns (None entries: gradient not requested); None if one has died."""
    out = []
    for r in refs:
        if r is None:
            continue
        p_ = r()
        if p_ is None:
            return None
        out.append(p_)
    return out or None


class ConvLayerFn(torch.autograd.Function):
    """One reference conv layer (causal / strided / transposed), channels-last."""

    @staticmethod
    def forward(ctx, x, w, b, kind, stride, dil, *out_float):
        # x: (B, T, Cin) contiguous in compute dtype; out_float (optional, True):
        # an fp32 output from a bf16 layer (the epilogue rounds to fp32 instead
        # of bf16; the backward takes the fp32 gradient to bf16 as a cast would)
        L.need_device(x, w)
        ctx.nextra = len(out_float)
        B, T_in, cin = x.shape
        if kind == PACK_CONVT:
            cout, k = w.shape[1], w.shape[2]
        else:
            cout, k = w.shape[0], w.shape[2]
        if kind == PACK_FWD and stride > 1:
            kind = PACK_FWD_STRIDED
            if k != 2 * stride:
                raise L.SelError(f"sel: strided CausalConv1d needs kernel_size == 2*stride (got {k}, {stride})")
        desc, T_out, c_out = _layer_desc(kind, B, T_in, cin, cout, k, stride, dil, b is not None)
        wp, wd = PACKS.get(kind, w, stride, x.dtype)
        bias = b.detach().contiguous().float() if b is not None else None
        y = prim(desc, x, wp, bias=bias, out_dtype=torch.float32 if out_float and out_float[0] else None)
        ctx.save_for_backward(x, wp, wd)
        ctx.meta = (desc, kind, stride, tuple(w.shape), b is not None)
        ctx.prefs = (weakref.ref(w), weakref.ref(b) if b is not None else None)
        return y.view(B, T_out, c_out)

    @staticmethod
    def backward(ctx, gy):
        x, wp, wd = ctx.saved_tensors
        desc, kind, stride, w_shape, has_bias = ctx.meta
        gy = gy.contiguous()
        if gy.dtype != x.dtype:
            gy = cast(gy, x.dtype)
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            gx = prim(desc.adjoint(), gy, wd)
            if desc.pad_mode == PAD_REPLICATE:
                L.call("sel_conv_replicate_fix", ctypes.byref(desc), _code(gy.dtype), L.ptr(gy), L.ptr(wp),
                       L.ptr(gx), L.stream())
            gx = gx.view(x.shape)
        if ctx.needs_input_grad[1] or (has_bias and ctx.needs_input_grad[2]):
            want_b = has_bias and ctx.needs_input_grad[2]
            params = _live(ctx.prefs[0], ctx.prefs[1] if want_b else None) if ctx.needs_input_grad[1] else None
            gw, gb = wgrad_torch(desc, gy, x, kind, w_shape, stride, want_b, params)
            if not ctx.needs_input_grad[1]:
                gw = None
        return (gx, gw, gb, None, None, None) + (None,) * ctx.nextra


# fused residual unit (sel_resunit_fwd / sel_resunit_bwd): ON by default at 32
# channels (register-resident 1x1, k_ru32_fwd / k_ru32_bwd) and for the
# 64-channel forward (k_ru64_fwd: the 1x1's h fragments exchanged between the
# two slice waves through LDS); SEL_RU_FUSED=0 turns every fused path off
RU_FUSED = os.environ.get("SEL_RU_FUSED", "")


def _ru_shape_ok(d1, dtype):
    """Mirror of the C side's eligibility (conv.hip ru_fused_ok)."""
    return (dtype == torch.bfloat16 and d1.C == d1.N and d1.C in (32, 64) and d1.K == 7
            and d1.pad == 6 * d1.dil and d1.pad_mode == PAD_ZERO and d1.in_elu == 1 and 6 * d1.dil <= 64
            and d1.bias_period in (0, d1.N))


def ru_fused_ok(d1, dtype):
    """Fused residual-unit forward for this conv1 descriptor?"""
    # SEL_RU_FUSED=32: the 32-channel unit only (A/B of the 64-channel forward)
    return RU_FUSED != "0" and _ru_shape_ok(d1, dtype) and (RU_FUSED != "32" or d1.C == 32)


WSS_PW_KID = 94 * 10 ** 7 + 128 * 10 ** 4 + 16 * 10 + 7   # k_conv_wss<7, 16, 128> (fwd_kernel_name)


def ru128_fused_ok(d1, dtype):
    """The 128-channel unit's forward as one k_conv_wss launch with the 1x1 in
    its epilogue (conv_wss.hip PW, conv.hip sel_resunit_fwd): where conv1 itself
    runs on the (16, 128) tile; tune key 69 = 1 turns it off."""
    if not (RU_FUSED != "0" and dtype == torch.bfloat16 and d1.C == d1.N == 128 and d1.K == 7
            and d1.pad == 6 * d1.dil and d1.pad_mode == PAD_ZERO and d1.in_elu == 1
            and d1.bias_period in (0, d1.N) and _tune_value(69) != 1):
        return False
    kid = L.lib().sel_conv_fwd_kernel_id(ctypes.byref(d1), _code(dtype), _code(dtype), 0)
    return kid == WSS_PW_KID


def ru_bwd_fused_ok(d1, dtype):
    """Fused residual-unit backward (k_ru32_bwd / k_ru64_bwd)?"""
    # SEL_RU_FUSED=32: the 32-channel unit only (A/B of the 64-channel kernels)
    return RU_FUSED != "0" and _ru_shape_ok(d1, dtype) and (RU_FUSED != "32" or d1.C == 32)


def resunit_bwd(d1, gf, h, xf, wd1, wd2, want_gh):
    """gx (and gh = (W2^T g) * ELU'(h) when want_gh) of a 32-channel residual unit
    in one launch; all (rows, 32) bf16."""
    gx = torch.empty_like(xf)
    gh = torch.empty_like(xf) if want_gh else None
    L.call("sel_resunit_bwd", ctypes.byref(d1), _code(xf.dtype), L.ptr(gf), L.ptr(h), L.ptr(xf), L.ptr(wd1),
           L.ptr(wd2), L.ptr(gh), L.ptr(gx), L.stream(), meta=lambda: _ru_bwd_meta(d1, xf, want_gh))
    return gx, gh


def _tune_value(key):
    """Current value of a sel_tune knob (read-only: no window in which another
    thread's dispatch could see it changed)."""
    return L.lib().sel_tune_get(key)


def _ru_bwd_meta(d1, xf, want_gh, wgrad=False):
    """Algorithmic bytes: read g, h, x once, write gx (and gh); flops of the two
    adjoints (and of the two weight gradients)."""
    es = xf.element_size()
    nbytes = (4 + int(want_gh)) * d1.rows * d1.C * es
    flops = 2.0 * d1.rows * d1.N * d1.C * (d1.K + 1) * (2 if wgrad else 1)
    if wgrad:
        return ("k_ru32_bwdw<128>" if d1.C == 32 else "k_ru64_bwdw<128>"), nbytes, flops
    if d1.C == 64 and not want_gh and _tune_value(41) == 1:
        return "k_ru64_bwdw<128, false>", nbytes, flops
    return ("k_ru32_bwd<128>" if d1.C == 32 else "k_ru64_bwd<128>"), nbytes, flops


# fused backward with both weight gradients (k_ru32_bwdw / k_ru64_bwdw);
# SEL_RU_WGRAD=0: off, =32: the 32-channel unit only (A/B of the 64-channel kernel)
RU_WGRAD = os.environ.get("SEL_RU_WGRAD", "1")


def ru_wgrad_fused_ok(d1, dtype):
    """Fused residual-unit backward with both weight gradients for this conv1?"""
    return (RU_WGRAD != "0" and ru_bwd_fused_ok(d1, dtype) and (d1.C == 32 or RU_WGRAD != "32"))


def resunit_bwd_wgrad(d1, gf, h, xf, wd1, wd2, s1, s2, want_b1, want_b2, params1, params2):
    """gx and both weight gradients of a 32- or 64-channel residual unit: ONE
    launch (k_ru32_bwdw / k_ru64_bwdw: gh, gx, and per-block partials of conv1
    and the 1x1), then the
    block-order reduction into the torch layouts, deferred to the end of the
    backward like wgrad_torch's when the parameters allow it (params1 / params2:
    the (weight, bias) leaves receiving gw1, gb1 / gw2, gb2, or None)."""
    lib = L.lib()
    ns = lib.sel_resunit_wgrad_splits(ctypes.byref(d1), _code(xf.dtype))
    if ns <= 0:
        raise L.SelError(f"sel_resunit_wgrad_splits failed ({ns}): {lib.sel_last_error().decode()}")
    N = d1.N
    nw1, nw2 = N * d1.K * d1.C, N * N
    n1 = ns * (nw1 + N)
    ws = torch.empty(n1 + ns * (nw2 + N), dtype=torch.float32, device=xf.device)
    gx = torch.empty_like(xf)
    st = L.stream()
    L.call("sel_resunit_bwd_wgrad", ctypes.byref(d1), _code(xf.dtype), L.ptr(gf), L.ptr(h), L.ptr(xf), L.ptr(wd1),
           L.ptr(wd2), L.ptr(gx), ctypes.c_void_p(ws.data_ptr()), ctypes.c_void_p(ws.data_ptr() + 4 * n1), ns, st,
           meta=lambda: _ru_bwd_meta(d1, xf, False, wgrad=True))
    out, jobs = [], []
    for (shape, want_b, params, off, nw, k) in ((s1, want_b1, params1, 0, nw1, d1.K), (s2, want_b2, params2, n1, nw2, 1)):
        defer = params is not None and len(params) == 1 + int(want_b) and _can_defer(params) and _queue_flush()
        if defer:
            gw = _grad_out(params[0], shape, xf.device)
            gb = _grad_out(params[1], (N,), xf.device) if want_b else None
        else:
            gw = torch.empty(shape, dtype=torch.float32, device=xf.device)
            gb = torch.empty(N, dtype=torch.float32, device=xf.device) if want_b else None
        job = _WgradJob(ws.data_ptr() + 4 * off, gw.data_ptr(), gb.data_ptr() if gb is not None else None, nw, ns, N,
                        N, PACK_FWD, shape[0], shape[1], k, 1)
        if defer:
            _defer(job, ws, params, gw, gb, st)
        else:
            jobs.append(job)
        out += [gw, gb]
    if jobs:
        arr = (_WgradJob * len(jobs))(*jobs)
        L.call("sel_wgrad_finish_many", ctypes.cast(arr, ctypes.c_void_p), len(jobs), st)
    return (gx, *out)


def resunit_fwd(d1, xf, wp1, b1, wp2, b2):
    """h = conv1(ELU(x)), out = x + conv1x1(ELU(h)) in one launch (both (rows, C) bf16)."""
    h = torch.empty((d1.rows, d1.N), dtype=xf.dtype, device=xf.device)
    out = torch.empty_like(h)
    L.call("sel_resunit_fwd", ctypes.byref(d1), _code(xf.dtype), L.ptr(xf), L.ptr(wp1), L.ptr(b1), L.ptr(wp2),
           L.ptr(b2), L.ptr(h), L.ptr(out), L.stream(), meta=lambda: _ru_meta(d1, xf, wp1, wp2))
    return h, out


def _ru_meta(d1, xf, wp1, wp2):
    """Algorithmic bytes: read x once, write h and out, read both packed weights."""
    es = xf.element_size()
    nbytes = 3 * d1.rows * d1.C * es + (wp1.numel() + wp2.numel()) * es
    flops = 2.0 * d1.rows * d1.N * d1.C * (d1.K + 1)
    # (the 32-channel unit's tile rows: 256, or 128 under tune key 56 = 1)
    if d1.C == 128:   # k_conv_wss PW: x is read twice (the DMA ring and the residual)
        return "k_conv_wss<7, 16, 128, bf16, PW>", nbytes + d1.rows * d1.C * es, flops
    tag = f"k_ru32_fwd<{128 if _tune_value(56) == 1 else 256}>" if d1.C == 32 else "k_ru64_fwd<128>"
    return tag, nbytes, flops


class ResidualUnitFn(torch.autograd.Function):
    """x + conv1x1(ELU(causal_conv_k(ELU(x)))) fused into two primitive calls
    forward and four backward (residual_unit.py:43-46).  `pad` (optional): the
    conv's left zero pad, (k-1)*dil causal by default; the noncausal unit
    (residual_unit.py:20-46) passes (k-1)//2*dil and runs the unfused kernels."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, dil, pad=None):
        L.need_device(x, w1, w2)
        B, T, C = x.shape
        k = w1.shape[2]
        cm = w1.shape[0]
        pad = (k - 1) * dil if pad is None else pad
        d1 = ConvDesc(B * T, T, C, cm, k, dil, pad, PAD_ZERO, 1, cm if b1 is not None else 0)
        d2 = ConvDesc(B * T, T, cm, w2.shape[0], 1, 1, 0, PAD_ZERO, 1, w2.shape[0] if b2 is not None else 0)
        if w2.shape[0] != C:
            raise L.SelError("residual unit needs out_channels == in_channels")
        wp1, wd1 = PACKS.get(PACK_FWD, w1, 1, x.dtype)
        wp2, wd2 = PACKS.get(PACK_FWD, w2, 1, x.dtype)
        bb1 = b1.detach().float().contiguous() if b1 is not None else None
        bb2 = b2.detach().float().contiguous() if b2 is not None else None
        xf = x.view(B * T, C)
        if ru_fused_ok(d1, x.dtype) or ru128_fused_ok(d1, x.dtype):
            h, out = resunit_fwd(d1, xf, wp1, bb1, wp2, bb2)
        else:
            h = prim(d1, xf, wp1, bias=bb1)
            out = prim(d2, h, wp2, bias=bb2, res=xf)
        ctx.save_for_backward(x, h, wd1, wd2)
        ctx.meta = (d1, d2, tuple(w1.shape), tuple(w2.shape))
        ctx.prefs = tuple(weakref.ref(p_) if p_ is not None else None for p_ in (w1, b1, w2, b2))
        return out.view(B, T, C)

    @staticmethod
    def backward(ctx, g):
        x, h, wd1, wd2 = ctx.saved_tensors
        d1, d2, s1, s2 = ctx.meta
        B, T, C = x.shape
        g = g.contiguous()
        if g.dtype != x.dtype:
            g = cast(g, x.dtype)
        gf = g.view(B * T, C)
        xf = x.view(B * T, C)
        need_w1 = ctx.needs_input_grad[1] or ctx.needs_input_grad[2]
        need_w2 = ctx.needs_input_grad[3] or ctx.needs_input_grad[4]
        gx = None
        pr = ctx.prefs
        if ctx.needs_input_grad[0] and need_w1 and need_w2 and ru_wgrad_fused_ok(d1, x.dtype):
            # one launch: gx and both weight gradients (k_ru32_bwdw / k_ru64_bwdw)
            want_b1 = d1.bias_period > 0 and ctx.needs_input_grad[2]
            want_b2 = d2.bias_period > 0 and ctx.needs_input_grad[4]
            p1 = _live(pr[0], pr[1] if want_b1 else None) if ctx.needs_input_grad[1] else None
            p2 = _live(pr[2], pr[3] if want_b2 else None) if ctx.needs_input_grad[3] else None
            gx, gw1, gb1, gw2, gb2 = resunit_bwd_wgrad(d1, gf, h, xf, wd1, wd2, s1, s2, want_b1, want_b2, p1, p2)
            return (gx.view(B, T, C), gw1 if ctx.needs_input_grad[1] else None, gb1,
                    gw2 if ctx.needs_input_grad[3] else None, gb2, None, None)
        if ctx.needs_input_grad[0] and ru_bwd_fused_ok(d1, x.dtype):
            # one launch: gh = (W2^T g) * ELU'(h) and gx = g + conv_adjoint(gh) * ELU'(x)
            gx, gh = resunit_bwd(d1, gf, h, xf, wd1, wd2, need_w1)
            gx = gx.view(B, T, C)
        else:
            # dL/dh = (W2^T g) * ELU'(h)
            gh = prim(d2.adjoint(), gf, wd2, aux=h)
        gw1 = gb1 = gw2 = gb2 = None
        if ctx.needs_input_grad[3] or ctx.needs_input_grad[4]:
            want_b = d2.bias_period > 0 and ctx.needs_input_grad[4]
            params = _live(pr[2], pr[3] if want_b else None) if ctx.needs_input_grad[3] else None
            gw2, gb2 = wgrad_torch(d2, gf, h, PACK_FWD, s2, 1, want_b, params)
            gw2 = gw2 if ctx.needs_input_grad[3] else None
        if ctx.needs_input_grad[0] and gx is None:
            # dL/dx = g + (conv_adjoint(gh)) * ELU'(x)
            gx = prim(d1.adjoint(), gh, wd1, aux=xf, res=gf).view(B, T, C)
        if need_w1:
            want_b = d1.bias_period > 0 and ctx.needs_input_grad[2]
            params = _live(pr[0], pr[1] if want_b else None) if ctx.needs_input_grad[1] else None
            gw1, gb1 = wgrad_torch(d1, gh, xf, PACK_FWD, s1, 1, want_b, params)
            gw1 = gw1 if ctx.needs_input_grad[1] else None
        return gx, gw1, gb1, gw2, gb2, None, None
