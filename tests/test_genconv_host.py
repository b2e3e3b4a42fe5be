"""Host logic of sel.genconv (the re-indexing that lowers any Conv1d /
ConvTranspose1d onto the stride-1 primitive), checked on CPU: the primitive's
entry points are replaced by a torch statement of their documented contract
(include/sel.h sel_conv_fwd / sel_conv_wgrad: y[r] = b + sum_k W[k] x[r + k*dil
- pad] within a sequence), so only the folding, padding, cropping, tap-group
and block-diagonal logic is under test here; the kernels themselves are
covered against the reference fixtures in tests/test_gpu_general.py."""
import pytest
import torch
import torch.nn.functional as F

from sel import convops as CO
from sel import genconv as GC


def _x3(desc, x):
    return x.reshape(desc.rows // desc.T, desc.T, -1).transpose(1, 2)


def _prim(desc, x, wp, bias=None, aux=None, res=None, out_dtype=None):
    assert aux is None and res is None and desc.in_elu == 0
    assert 0 <= desc.pad and (desc.K - 1) * desc.dil <= 512
    xt = F.pad(_x3(desc, x), (desc.pad, max((desc.K - 1) * desc.dil - desc.pad, 0)))
    y = F.conv1d(xt, wp.permute(0, 2, 1), dilation=desc.dil)[:, :, :desc.T]
    if bias is not None:
        y = y + bias.repeat(desc.N // bias.numel()).view(1, -1, 1)
    return y.transpose(1, 2).reshape(desc.rows, desc.N)


def _wgrad(desc, gy, x, want_b):
    assert desc.K <= 8, "sel_conv_wgrad takes K <= 8"
    xt = F.pad(_x3(desc, x), (desc.pad, (desc.K - 1) * desc.dil))
    gyt = _x3(desc, gy)
    gw = torch.stack([torch.einsum("bnt,bct->nc", gyt, xt[:, :, k * desc.dil:k * desc.dil + desc.T])
                      for k in range(desc.K)], 1)
    return gw, (gyt.sum((0, 2)) if want_b else None)


@pytest.fixture
def emulated(monkeypatch):
    monkeypatch.setattr(CO, "pack", lambda kind, w, stride, dtype: w.detach().permute(0, 2, 1).contiguous())
    monkeypatch.setattr(CO, "pack_dgrad", lambda wp: wp.flip(1).permute(2, 1, 0).contiguous())
    monkeypatch.setattr(CO, "prim", _prim)
    monkeypatch.setattr(CO, "wgrad", _wgrad)
    monkeypatch.setattr(CO, "unpack", lambda kind, gwp, shape, stride: gwp.permute(0, 2, 1).contiguous())
    monkeypatch.setattr(CO, "cast", lambda x, dt: x.to(dt))


def _check(fn, ref, x, w, b):
    xs = [t.clone().double().requires_grad_(True) if t is not None else None for t in (x, w, b)]
    xr = [t.clone().double().requires_grad_(True) if t is not None else None for t in (x, w, b)]
    y = fn(*xs)
    yr = ref(*xr)
    assert y.shape == yr.shape, (y.shape, yr.shape)
    torch.testing.assert_close(y, yr, rtol=1e-10, atol=1e-10)
    r = torch.randn_like(yr)
    (y * r).sum().backward()
    (yr * r).sum().backward()
    for a, c in zip(xs, xr):
        if a is not None:
            torch.testing.assert_close(a.grad, c.grad, rtol=1e-10, atol=1e-10)


CONV = [  # Cin, Cout, k, stride, padding, dilation, groups, T
    (3, 5, 7, 1, 3, 1, 1, 40), (4, 6, 6, 3, 2, 1, 1, 61), (4, 4, 5, 2, 0, 2, 2, 33),
    (8, 8, 41, 4, 20, 1, 4, 90), (2, 3, 3, 1, 6, 1, 1, 20), (6, 6, 4, 5, 7, 3, 3, 50),
    (3, 4, 12, 1, 2, 1, 1, 30),
    # edge cases: one input sample with a stride, a 512-row halo (the primitive's
    # bound), a 1-tap strided conv
    (1, 1, 3, 2, 1, 1, 1, 1), (5, 3, 9, 1, 256, 64, 1, 600), (2, 2, 1, 3, 0, 1, 1, 10)]


@pytest.mark.parametrize("cfg", CONV)
def test_conv1d_lowering(emulated, cfg):
    ci, co, k, s, p, dl, g, t = cfg
    torch.manual_seed(0)
    x, w, b = torch.randn(2, t, ci), torch.randn(co, ci // g, k), torch.randn(co)
    _check(lambda x, w, b: GC.conv1d(x, w, b, s, p, dl, g),
           lambda x, w, b: F.conv1d(x.transpose(1, 2), w, b, s, p, dl, g).transpose(1, 2), x, w, b)


def test_causal_conv1d_lowering(emulated):
    torch.manual_seed(1)
    for ci, co, k, s, dl, g, t in [(4, 4, 7, 1, 2, 2, 30), (3, 5, 4, 3, 1, 1, 31), (6, 3, 3, 2, 1, 3, 9)]:
        x, w, b = torch.randn(2, t, ci), torch.randn(co, ci // g, k), torch.randn(co)
        _check(lambda x, w, b: GC.conv1d(x, w, b, s, (k - 1) * dl, dl, g, (t - 1) // s + 1),
               lambda x, w, b: F.conv1d(F.pad(x.transpose(1, 2), ((k - 1) * dl, 0)), w, b, s, 0, dl, g)
               .transpose(1, 2), x, w, b)


CONVT = [  # Cin, Cout, k, stride, padding, output_padding, groups, T
    (4, 3, 10, 5, 3, 1, 1, 12), (4, 6, 8, 4, 2, 0, 1, 9), (4, 6, 5, 3, 1, 2, 2, 10),
    (3, 2, 3, 1, 0, 0, 1, 7), (2, 2, 7, 3, 3, 0, 1, 5), (3, 3, 3, 2, 0, 1, 1, 6),
    # edge cases: one input sample, a 1-tap transposed conv with output padding
    (2, 3, 4, 2, 0, 1, 1, 1), (3, 3, 1, 3, 0, 2, 1, 4)]


@pytest.mark.parametrize("cfg", CONVT)
def test_conv_transpose1d_lowering(emulated, cfg):
    ci, co, k, s, p, op, g, t = cfg
    torch.manual_seed(2)
    x, w, b = torch.randn(2, t, ci), torch.randn(ci, co // g, k), torch.randn(co)
    _check(lambda x, w, b: GC.conv_transpose1d(x, w, b, s, p, op, g),
           lambda x, w, b: F.conv_transpose1d(x.transpose(1, 2), w, b, s, p, op, g).transpose(1, 2), x, w, b)
