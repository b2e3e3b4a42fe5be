"""Adam for the generator / discriminator updates (trainer/trainerGAN.py:271-281
`optimizer.step()`; the reference builds torch.optim.Adam from the config's
*_optimizer_params): the update of every parameter tensor in one HIP launch
(sel_adam_step_many) instead of torch's fused multi-tensor kernel, which
reached about 45% of the HBM rate at C3 (50 us per step for the encoder).

torch.optim.Adam semantics and state layout ("step", "exp_avg", "exp_avg_sq"
per parameter; state_dict / load_state_dict interchangeable with torch's Adam):
L2 weight decay, bias corrections from each parameter's own step count.  The
options the product path does not use (amsgrad, maximize, differentiable,
non-fp32 or sparse gradients) are refused; `adam(...)` builds torch's Adam for
those and whenever SEL_ADAM=torch.

capturable=True (the role of torch's capturable Adam): every parameter group
keeps ONE step count and its learning rate in device memory
(sel_adam_step_many_dev advances the count and derives the bias corrections on
the device), so a step captured in a HIP graph (trainer.graph) is correct on
every replay.  A changed group["lr"] (an LR scheduler) reaches the device copy
at the next eager step() or through sync_lr(); the parameters of a group share
its step count (their state["step"] is that one device tensor).
"""
import ctypes
import math
import os

import torch

from . import _lib as L


class _AdamTensor(ctypes.Structure):
    """sel_adam_tensor (include/sel.h)."""
    _fields_ = [("p", ctypes.c_void_p), ("g", ctypes.c_void_p), ("m", ctypes.c_void_p), ("v", ctypes.c_void_p),
                ("n", ctypes.c_int64)]


class Adam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, amsgrad=False, *,
                 maximize=False, foreach=None, capturable=False, differentiable=False, fused=None):
        if amsgrad or maximize or differentiable:
            raise NotImplementedError("sel.optim.Adam: amsgrad / maximize / differentiable "
                                      "are not supported (use torch.optim.Adam)")
        if not 0.0 <= lr or not 0.0 <= eps or not 0.0 <= weight_decay:
            raise ValueError(f"invalid Adam hyper-parameters lr={lr} eps={eps} weight_decay={weight_decay}")
        if not (0.0 <= betas[0] < 1.0 and 0.0 <= betas[1] < 1.0):
            raise ValueError(f"invalid betas {betas}")
        super().__init__(params, dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay, amsgrad=False,
                                      maximize=False, foreach=None, capturable=bool(capturable),
                                      differentiable=False, fused=None))
        self._dev = {}  # capturable: id(group) -> (lr tensor, step tensor, consts tensor, host lr)

    def _group_dev(self, group, device):
        d = self._dev.get(id(group))
        if d is None:
            lr = torch.full((1,), float(group["lr"]), dtype=torch.float32, device=device)
            d = [lr, torch.zeros((), dtype=torch.float32, device=device),
                 torch.zeros(2, dtype=torch.float32, device=device), float(group["lr"])]
            self._dev[id(group)] = d
        return d

    def sync_lr(self):
        """Copy changed group learning rates to their device copies (eager only)."""
        for group in self.param_groups:
            d = self._dev.get(id(group))
            if d is not None and d[3] != float(group["lr"]):
                d[0].fill_(float(group["lr"]))
                d[3] = float(group["lr"])

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            if group["capturable"]:
                self._step_dev(group)
                continue
            b1, b2 = group["betas"]
            by_step = {}
            for p in group["params"]:
                if p.grad is None:
                    continue
                g = p.grad
                if g.is_sparse or p.dtype != torch.float32 or g.dtype != torch.float32 or not p.is_cuda:
                    raise NotImplementedError("sel.optim.Adam: dense fp32 device parameters only")
                if not g.is_contiguous() or not p.is_contiguous():
                    raise NotImplementedError("sel.optim.Adam: contiguous parameters and gradients only")
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = torch.tensor(0.0, dtype=torch.float32)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["step"] += 1
                by_step.setdefault(int(st["step"].item()), []).append((p, g, st))
            for t, items in by_step.items():
                step_size = group["lr"] / (1.0 - b1 ** t)
                bc2_sqrt = math.sqrt(1.0 - b2 ** t)
                arr = (_AdamTensor * len(items))(*[
                    _AdamTensor(p.data_ptr(), g.data_ptr(), st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr(),
                                p.numel()) for p, g, st in items])
                L.call("sel_adam_step_many", ctypes.cast(arr, ctypes.c_void_p), len(items), float(b1), float(b2),
                       float(group["eps"]), float(group["weight_decay"]), float(step_size), float(bc2_sqrt),
                       L.stream())
        return loss

    def _step_dev(self, group):
        b1, b2 = group["betas"]
        items = []
        for p in group["params"]:
            if p.grad is None:
                continue
            g = p.grad
            if g.is_sparse or p.dtype != torch.float32 or g.dtype != torch.float32 or not p.is_cuda:
                raise NotImplementedError("sel.optim.Adam: dense fp32 device parameters only")
            if not g.is_contiguous() or not p.is_contiguous():
                raise NotImplementedError("sel.optim.Adam: contiguous parameters and gradients only")
            items.append((p, g))
        if not items:
            return
        d = self._group_dev(group, items[0][0].device)
        if not torch.cuda.is_current_stream_capturing():
            self.sync_lr()
        for p, _ in items:
            st = self.state[p]
            if len(st) == 0:
                st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            if st.get("step") is not d[1]:
                if "step" in st:  # a loaded state: the group's count takes it over
                    d[1].fill_(float(st["step"]))
                st["step"] = d[1]
        arr = (_AdamTensor * len(items))(*[
            _AdamTensor(p.data_ptr(), g.data_ptr(), self.state[p]["exp_avg"].data_ptr(),
                        self.state[p]["exp_avg_sq"].data_ptr(), p.numel()) for p, g in items])
        L.call("sel_adam_step_many_dev", ctypes.cast(arr, ctypes.c_void_p), len(items), float(b1), float(b2),
               float(group["eps"]), float(group["weight_decay"]), L.ptr(d[0]), L.ptr(d[1]), L.ptr(d[2]), L.stream())


def adam(params, **kw):
    """sel.optim.Adam where it applies (fp32 device parameters, the plain
    options), else torch.optim.Adam with the same arguments; SEL_ADAM=torch:
    always torch's (fused on the GPU, as the caller asked)."""
    params = list(params)
    plain = not any(kw.get(k) for k in ("amsgrad", "maximize", "differentiable"))
    on_gpu = all((p["params"][0] if isinstance(p, dict) else p).is_cuda for p in params[:1]) if params else False
    if os.environ.get("SEL_ADAM", "sel") != "torch" and plain and on_gpu:
        kw = {k: v for k, v in kw.items() if k not in ("fused", "foreach")}
        return Adam(params, **kw)
    return torch.optim.Adam(params, **kw)
