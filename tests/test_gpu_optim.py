"""sel.optim.Adam (sel_adam_step_many, the optimizer.step() of
trainer/trainerGAN.py:271-281) against torch.optim.Adam: same update rule and
state layout.  The arithmetic is torch's fused kernel's formula; the bias
corrections are computed on the host in double and the compilers contract
different products into fused multiply-adds, so results agree to a few fp32
ulps (moments: relative to their scale), not bit for bit."""
import copy

import pytest
import torch

from sel import optim as O

pytestmark = pytest.mark.gpu

SHAPES = [(64, 32, 7), (1,), (3, 5), (1023,), (256, 256, 7), (8, 1, 2)]


def _params(dev, seed):
    g = torch.Generator().manual_seed(seed)
    return [torch.randn(*s, generator=g).to(dev).requires_grad_(True) for s in SHAPES]


@pytest.mark.parametrize("kw", [dict(lr=1e-4, betas=(0.5, 0.9), weight_decay=0.0),
                                dict(lr=5e-5, weight_decay=1e-6), dict(lr=2e-4, betas=(0.8, 0.99), eps=1e-6)])
def test_sel_adam_matches_torch_adam(gpu, kw):
    a, b = _params(gpu, 1), _params(gpu, 1)
    # the reference's own optimizer: torch.optim.Adam with its defaults (foreach on
    # the GPU); torch's fused kernel applies the L2 decay with other roundings
    # (exp_avg_sq 1e-5 apart at weight_decay 1e-6)
    oa, ob = O.Adam(a, **kw), torch.optim.Adam(b, **kw)
    g = torch.Generator().manual_seed(7)
    for it in range(6):
        grads = [torch.randn(p.shape, generator=g).to(gpu) * (10.0 ** (it % 3 - 1)) for p in a]
        for p, q, gr in zip(a, b, grads):
            p.grad = gr.clone()
            q.grad = gr.clone()
        if it == 3:  # a parameter without a gradient this step keeps its own step count
            a[1].grad = None
            b[1].grad = None
        oa.step()
        ob.step()
        for p, q in zip(a, b):
            torch.testing.assert_close(p, q, rtol=2e-6, atol=1e-7)
    for p, q in zip(a, b):
        sa, sb = oa.state[p], ob.state[q]
        assert float(sa["step"]) == float(sb["step"])
        # moments: relative to their scale (a moment near 0 is a cancellation of
        # steps whose last bits depend on the fused-multiply-add contraction)
        for k in ("exp_avg", "exp_avg_sq"):
            torch.testing.assert_close(sa[k], sb[k], rtol=1e-6, atol=1e-6 * float(sb[k].abs().max()))


def test_sel_adam_state_dict_interchangeable_with_torch(gpu):
    kw = dict(lr=1e-3, betas=(0.5, 0.9))
    a, b = _params(gpu, 2), _params(gpu, 2)
    ob = torch.optim.Adam(b, **kw)
    g = torch.Generator().manual_seed(3)
    for _ in range(3):
        for p, q in zip(a, b):
            gr = torch.randn(p.shape, generator=g).to(gpu)
            p.grad, q.grad = gr.clone(), gr.clone()
        ob.step()
    with torch.no_grad():
        for p, q in zip(a, b):
            p.copy_(q)
    oa = O.Adam(a, **kw)
    # a deep copy: load_state_dict keeps the saved CPU step tensors, which both
    # optimizers would then increment in place
    oa.load_state_dict(copy.deepcopy(ob.state_dict()))
    for p, q in zip(a, b):
        gr = torch.randn(p.shape, generator=g).to(gpu)
        p.grad, q.grad = gr.clone(), gr.clone()
    oa.step()
    ob.step()
    for p, q in zip(a, b):
        torch.testing.assert_close(p, q, rtol=2e-6, atol=1e-7)
    sd = oa.state_dict()
    assert set(sd["state"][0]) == {"step", "exp_avg", "exp_avg_sq"}
