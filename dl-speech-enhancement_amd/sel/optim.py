"""Adam for the generator / discriminator updates (trainer/trainerGAN.py:271-281
`optimizer.step()`; the reference builds torch.optim.Adam from the config's
*_optimizer_params): the update of every parameter tensor in one HIP launch
(sel_adam_step_many) instead of torch's fused multi-tensor kernel, which
reached about 45% of the HBM rate at C3 (50 us per step for the encoder).

torch.optim.Adam semantics and state layout ("step", "exp_avg", "exp_avg_sq"
per parameter; state_dict / load_state_dict interchangeable with torch's Adam):
L2 weight decay, bias corrections from each parameter's own step count.  The
options the product path does not use (amsgrad, maximize, capturable,
differentiable, non-fp32 or sparse gradients) are refused; `adam(...)` builds
torch's Adam for those and whenever SEL_ADAM=torch.
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
        if amsgrad or maximize or capturable or differentiable:
            raise NotImplementedError("sel.optim.Adam: amsgrad / maximize / capturable / differentiable "
                                      "are not supported (use torch.optim.Adam)")
        if not 0.0 <= lr or not 0.0 <= eps or not 0.0 <= weight_decay:
            raise ValueError(f"invalid Adam hyper-parameters lr={lr} eps={eps} weight_decay={weight_decay}")
        if not (0.0 <= betas[0] < 1.0 and 0.0 <= betas[1] < 1.0):
            raise ValueError(f"invalid betas {betas}")
        super().__init__(params, dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay, amsgrad=False,
                                      maximize=False, foreach=None, capturable=False, differentiable=False,
                                      fused=None))

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
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


def adam(params, **kw):
    """sel.optim.Adam where it applies (fp32 device parameters, the plain
    options), else torch.optim.Adam with the same arguments; SEL_ADAM=torch:
    always torch's (fused on the GPU, as the caller asked)."""
    params = list(params)
    plain = not any(kw.get(k) for k in ("amsgrad", "maximize", "capturable", "differentiable"))
    on_gpu = all((p["params"][0] if isinstance(p, dict) else p).is_cuda for p in params[:1]) if params else False
    if os.environ.get("SEL_ADAM", "sel") != "torch" and plain and on_gpu:
        kw = {k: v for k, v in kw.items() if k not in ("fused", "foreach")}
        return Adam(params, **kw)
    return torch.optim.Adam(params, **kw)
