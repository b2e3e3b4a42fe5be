"""GPU parity of the conv-stack kernels (layers/conv_layer.py drop-ins, residual unit).

fp32 path (v_mfma_f32_16x16x4_f32, exact fp32 products, different summation
order than MKL-DNN): relative error <= 1e-5 on outputs, 1e-4 on gradients
(norm-wise), plus elementwise |a-b| <= 1e-4|b| + 1e-5 max|b|.
bf16 path (bf16 operands, fp32 accumulation): <= 2e-2 norm-wise relative.
"""
import numpy as np
import pytest
import torch

from conftest import golden

pytestmark = pytest.mark.gpu


def _np(t):
    return t.detach().float().cpu().numpy() if torch.is_tensor(t) else np.asarray(t)


def close(a, b, rtol=1e-4, floor=1e-5):
    a, b = _np(a).astype(np.float64), _np(b).astype(np.float64)
    assert a.shape == b.shape, (a.shape, b.shape)
    nb = np.linalg.norm(b) + 1e-30
    assert np.linalg.norm(a - b) <= rtol * nb, np.linalg.norm(a - b) / nb
    bad = np.abs(a - b) > rtol * np.abs(b) + floor * np.abs(b).max()
    assert not bad.any(), f"{bad.sum()} bad, worst {np.abs(a - b)[bad].max()}"


def nclose(a, b, rtol):
    a, b = _np(a).astype(np.float64), _np(b).astype(np.float64)
    assert a.shape == b.shape
    e = np.linalg.norm(a - b) / (np.linalg.norm(b) + 1e-30)
    assert e <= rtol, e


def _layer(name, cfg, g, dev):
    from layers.conv_layer import CausalConv1d, CausalConvTranspose1d
    if len(cfg) == 7:
        ci, co, k, s, d, hb, t = (int(v) for v in cfg)
        m = CausalConv1d(ci, co, k, stride=s, dilation=d, bias=bool(hb))
        p = m.conv
    else:
        ci, co, k, s, hb, t = (int(v) for v in cfg)
        m = CausalConvTranspose1d(ci, co, k, s, bias=bool(hb))
        p = m.deconv
    with torch.no_grad():
        p.weight.copy_(torch.from_numpy(g[f"{name}.w"]))
        if p.bias is not None:
            p.bias.copy_(torch.from_numpy(g[f"{name}.b"]))
    return m.to(dev), p


@pytest.mark.parametrize("name", ["first", "ru_d1", "ru_d3", "ru_d9", "down3", "down5", "proj", "last",
                                  "up5", "up3", "up4"])
def test_conv_layer_matches_reference_golden(gpu, name):
    g = golden("conv")
    m, p = _layer(name, g[f"{name}.cfg"], g, gpu)
    x = torch.from_numpy(g[f"{name}.x"]).to(gpu).requires_grad_(True)
    y = m(x)
    close(y, g[f"{name}.y"], 1e-5)
    y.backward(torch.from_numpy(g[f"{name}.gy"]).to(gpu))
    close(x.grad, g[f"{name}.gx"])
    close(p.weight.grad, g[f"{name}.gw"])
    if p.bias is not None:
        close(p.bias.grad, g[f"{name}.gb"])


def test_residual_unit_matches_reference_golden(gpu):
    from models.autoencoder.modules.residual_unit import CausalResidualUnit
    g = golden("conv")
    ru = CausalResidualUnit(8, 8, dilation=3)
    with torch.no_grad():
        ru.conv1.conv.weight.copy_(torch.from_numpy(g["ru.w1"]))
        ru.conv2.weight.copy_(torch.from_numpy(g["ru.w2"]))
    ru = ru.to(gpu)
    x = torch.from_numpy(g["ru.x"]).to(gpu).requires_grad_(True)
    y = ru(x)
    close(y, g["ru.y"], 1e-5)
    y.backward(torch.from_numpy(g["ru.gy"]).to(gpu))
    close(x.grad, g["ru.gx"])
    close(ru.conv1.conv.weight.grad, g["ru.gw1"])
    close(ru.conv2.weight.grad, g["ru.gw2"])


SHAPES = [
    # (kind, Cin, Cout, k, stride, dil, bias, B, T)   full-width AudioDec layers, short T
    ("conv", 32, 32, 7, 1, 9, False, 2, 600),
    ("conv", 64, 64, 7, 1, 3, False, 2, 320),
    ("conv", 256, 256, 7, 1, 9, False, 2, 80),
    ("conv", 512, 512, 7, 1, 1, False, 2, 20),
    ("conv", 512, 64, 3, 1, 1, False, 3, 20),
    ("conv", 32, 1, 7, 1, 1, False, 2, 300),
    ("conv", 1, 32, 7, 1, 1, False, 2, 300),
    ("conv", 32, 64, 6, 3, 1, True, 2, 600),
    ("conv", 256, 512, 10, 5, 1, True, 2, 100),
    ("convT", 512, 256, 10, 5, 1, True, 2, 16),
    ("convT", 64, 32, 6, 3, 1, True, 3, 100),
]


def _ref_and_dev(kind, ci, co, k, s, d, hb, B, T, dev, seed):
    from layers.conv_layer import CausalConv1d, CausalConvTranspose1d
    from oracle import ref_ops as R
    torch.manual_seed(seed)
    if kind == "conv":
        m = CausalConv1d(ci, co, k, stride=s, dilation=d, bias=hb)
        p = m.conv
        ref = lambda x, w, b: R.causal_conv1d(x, w, b, s, d)
    else:
        m = CausalConvTranspose1d(ci, co, k, s, bias=hb)
        p = m.deconv
        ref = lambda x, w, b: R.causal_conv_transpose1d(x, w, b, s)
    x = torch.randn(B, ci, T)
    w = p.weight.detach().clone().requires_grad_(True)
    b = p.bias.detach().clone().requires_grad_(True) if hb else None
    xr = x.clone().requires_grad_(True)
    yr = ref(xr, w, b)
    gy = torch.randn_like(yr)
    yr.backward(gy)
    return m.to(dev), p, x, gy, (yr, xr.grad, w.grad, b.grad if hb else None)


@pytest.mark.parametrize("shape", SHAPES, ids=[f"{s[0]}{s[1]}-{s[2]}k{s[3]}s{s[4]}d{s[5]}" for s in SHAPES])
def test_conv_layer_fp32_vs_oracle(gpu, shape):
    m, p, x, gy, (yr, gxr, gwr, gbr) = _ref_and_dev(*shape, gpu, seed=hash(shape) % 1000)
    xd = x.to(gpu).requires_grad_(True)
    y = m(xd)
    close(y, yr, 1e-5)
    y.backward(gy.to(gpu))
    close(xd.grad, gxr)
    close(p.weight.grad, gwr)
    if gbr is not None:
        close(p.bias.grad, gbr)


@pytest.mark.parametrize("shape", SHAPES[:4] + SHAPES[5:], ids=lambda s: f"{s[0]}{s[1]}-{s[2]}")
def test_conv_layer_bf16_vs_oracle(gpu, shape):
    from sel import convops as CO
    m, p, x, gy, (yr, gxr, gwr, gbr) = _ref_and_dev(*shape, gpu, seed=7)
    xd = x.to(gpu).requires_grad_(True)
    with CO.precision(torch.bfloat16):
        y = m(xd)
        assert y.dtype == torch.bfloat16
        nclose(y, yr, 2e-2)
        y.float().backward(gy.to(gpu))
    nclose(xd.grad, gxr, 2e-2)
    nclose(p.weight.grad, gwr, 2e-2)


def test_channels_last_views_flow_without_copies(gpu):
    from layers.conv_layer import CausalConv1d
    a = CausalConv1d(32, 32, 7, dilation=3).to(gpu)
    b = CausalConv1d(32, 64, 6, stride=3).to(gpu)
    x = torch.randn(2, 32, 600, device=gpu)
    y = a(x)
    assert y.shape == (2, 32, 600) and y.stride(1) == 1  # (B,C,T) view of (B,T,C)
    z = b(y)
    assert z.shape == (2, 64, 200) and z.stride(1) == 1


# C3 layer shapes (primitive form): C, N, K, dil, pad_mode, in_elu, bias, T
WGRAD_SHAPES = [(32, 32, 7, 9, 0, 1, 0, 2400), (32, 32, 1, 1, 0, 1, 0, 2400), (96, 64, 3, 1, 0, 0, 64, 800),
                (64, 64, 7, 3, 0, 1, 0, 800), (64, 64, 1, 1, 0, 1, 0, 800), (64, 96, 2, 1, 1, 0, 32, 800),
                (256, 128, 3, 1, 0, 0, 128, 200), (128, 128, 7, 9, 0, 1, 0, 200), (256, 256, 7, 1, 0, 1, 0, 40),
                (640, 256, 3, 1, 0, 0, 256, 40), (512, 1280, 2, 1, 1, 0, 256, 8), (32, 64, 7, 1, 0, 0, 0, 300),
                (1, 32, 7, 1, 0, 0, 0, 2400), (1, 32, 7, 1, 0, 1, 32, 2400), (1, 64, 3, 2, 0, 0, 0, 500)]


@pytest.mark.parametrize("shape", WGRAD_SHAPES)
def test_wgrad_kernels_agree(gpu, shape):
    """Every bf16 weight-gradient kernel (tune key 1: 0 = k_wgrad3, 1 = generic,
    2 = k_wgrad2) must give the same fp32 sums as the fp32 oracle of the same
    bf16 operands: 1e-5 norm-wise (fp32 accumulation, different orders)."""
    import ctypes
    from sel import _lib as L
    from sel import convops as CO
    C, N, K, dil, mode, elu, bias, T = shape
    B = 4
    pad = (K - 1) * dil if mode == 0 else 1
    d = CO.ConvDesc(B * T, T, C, N, K, dil, pad, mode, elu, bias)
    torch.manual_seed(C + N + K)
    x = (0.5 * torch.randn(B * T, C, device=gpu)).to(torch.bfloat16)
    g = (0.5 * torch.randn(B * T, N, device=gpu)).to(torch.bfloat16)
    # fp64 reference of the same bf16 operands
    xa = x.double().view(B, T, C)
    if elu:
        xa = torch.nn.functional.elu(xa.float()).to(torch.bfloat16).double()
    ga = g.double().view(B, T, N)
    ref = torch.zeros(N, K, C, dtype=torch.float64, device=gpu)
    for k in range(K):
        idx = torch.arange(T, device=gpu) + k * dil - pad
        if mode == 0:
            ok = (idx >= 0) & (idx < T)
            xs = torch.zeros(B, T, C, dtype=torch.float64, device=gpu)
            xs[:, ok] = xa[:, idx[ok]]
        else:
            xs = xa[:, idx.clamp(0, T - 1)]
        ref[:, k, :] = torch.einsum("btn,btc->nc", ga, xs)
    bref = ga.sum((0, 1)).view(-1, bias).sum(0) if bias else None
    lib = L.lib()
    for variant in (0, 1, 2):
        prev = lib.sel_tune(1, variant)
        try:
            gw, gb = CO.wgrad(d, g, x, bool(bias))
        finally:
            lib.sel_tune(1, prev)
        e = ((gw.double() - ref).norm() / ref.norm()).item()
        assert e < 2e-3 if elu else e < 1e-5, (variant, e)
        if bias:
            eb = ((gb.double() - bref).norm() / bref.norm()).item()
            assert eb < 1e-5, (variant, eb)


@pytest.mark.parametrize("shape", WGRAD_SHAPES)
def test_wgrad_fp32_kernels_agree(gpu, shape):
    """fp32 weight gradients: the sample-tiled k_wgrad_f32 (default where it
    applies) and the generic k_conv_wgrad (tune key 54 = 1) against fp64 of the
    same fp32 operands, 1e-5 norm-wise (fp32 products and sums, other orders);
    includes ragged tiles (T % 64 != 0), replicate padding and the C = 1 layers."""
    from sel import _lib as L
    from sel import convops as CO
    C, N, K, dil, mode, elu, bias, T = shape
    B = 3
    T = T + 13  # ragged last tile of every sample
    pad = (K - 1) * dil if mode == 0 else 1
    d = CO.ConvDesc(B * T, T, C, N, K, dil, pad, mode, elu, bias)
    torch.manual_seed(C + N + K + 1)
    x = 0.5 * torch.randn(B * T, C, device=gpu)
    g = 0.5 * torch.randn(B * T, N, device=gpu)
    xa = x.double().view(B, T, C)
    if elu:
        xa = torch.where(xa > 0, xa, torch.expm1(xa))
    ga = g.double().view(B, T, N)
    ref = torch.zeros(N, K, C, dtype=torch.float64, device=gpu)
    for k in range(K):
        idx = torch.arange(T, device=gpu) + k * dil - pad
        if mode == 0:
            ok = (idx >= 0) & (idx < T)
            xs = torch.zeros(B, T, C, dtype=torch.float64, device=gpu)
            xs[:, ok] = xa[:, idx[ok]]
        else:
            xs = xa[:, idx.clamp(0, T - 1)]
        ref[:, k, :] = torch.einsum("btn,btc->nc", ga, xs)
    bref = ga.sum((0, 1)).view(-1, bias).sum(0) if bias else None
    lib = L.lib()
    for variant in (0, 1):
        prev = lib.sel_tune(54, variant)
        try:
            gw, gb = CO.wgrad(d, g, x, bool(bias))
        finally:
            lib.sel_tune(54, prev)
        e = ((gw.double() - ref).norm() / ref.norm()).item()
        assert e < 1e-5, (variant, e)
        if bias:
            eb = ((gb.double() - bref).norm() / bref.norm()).item()
            assert eb < 1e-5, (variant, eb)


@pytest.mark.parametrize("shape", WGRAD_SHAPES)
def test_fwd_fp32_kernels_agree(gpu, shape):
    """fp32 forward primitive: the sample-tiled k_conv_fwd_f32 (default where it
    applies) and the generic k_conv_fwd (tune key 55 = 1) against fp64 of the
    same operands with bias, ELU'(aux) and residual epilogues: 1e-5 norm-wise;
    ragged tiles (T % 64 != 0), replicate padding and the C = 1 layers."""
    from sel import _lib as L
    from sel import convops as CO
    C, N, K, dil, mode, elu, bias, T = shape
    B = 3
    T = T + 13
    pad = (K - 1) * dil if mode == 0 else 1
    d = CO.ConvDesc(B * T, T, C, N, K, dil, pad, mode, elu, N if bias else 0)
    torch.manual_seed(C + N + K + 2)
    x = 0.5 * torch.randn(B * T, C, device=gpu)
    wp = 0.2 * torch.randn(N, K, C, device=gpu)
    b = torch.randn(N, device=gpu) if bias else None
    aux = torch.randn(B * T, N, device=gpu)
    res = torch.randn(B * T, N, device=gpu)
    xa = x.double().view(B, T, C)
    if elu:
        xa = torch.where(xa > 0, xa, torch.expm1(xa))
    ref = torch.zeros(B, T, N, dtype=torch.float64, device=gpu)
    for k in range(K):
        idx = torch.arange(T, device=gpu) + k * dil - pad
        if mode == 0:
            ok = (idx >= 0) & (idx < T)
            xs = torch.zeros(B, T, C, dtype=torch.float64, device=gpu)
            xs[:, ok] = xa[:, idx[ok]]
        else:
            xs = xa[:, idx.clamp(0, T - 1)]
        ref += torch.einsum("btc,nc->btn", xs, wp[:, k, :].double())
    if bias:
        ref += b.double()
    ref = ref.view(B * T, N)
    refe = ref * torch.where(aux.double() > 0, 1.0, torch.exp(aux.double())) + res.double()
    lib = L.lib()
    for variant in (0, 1):
        prev = lib.sel_tune(55, variant)
        try:
            y = CO.prim(d, x, wp, bias=b)
            ye = CO.prim(d, x, wp, bias=b, aux=aux, res=res)
        finally:
            lib.sel_tune(55, prev)
        for got, want in ((y, ref), (ye, refe)):
            e = ((got.double() - want).norm() / want.norm()).item()
            assert e < 1e-5, (variant, e)


@pytest.mark.parametrize("C,N,K,dil,elu,aux,res", [(1, 32, 7, 1, 0, 0, 0), (1, 32, 7, 1, 1, 1, 1), (1, 64, 3, 2, 0, 1, 0)])
def test_single_channel_kernel_matches_generic(gpu, C, N, K, dil, elu, aux, res):
    """The streaming C=1 kernel (tune key 3 = 0) against the generic implicit-GEMM
    kernel on the same bf16 operands: both accumulate the K products in fp32, the
    epilogue ELU' uses the same hardware exp -> within one bf16 ulp (4e-3 rel)."""
    from sel import _lib as L
    from sel import convops as CO
    B, T = 3, 1000
    d = CO.ConvDesc(B * T, T, C, N, K, dil, (K - 1) * dil, CO.PAD_ZERO, elu, N)
    torch.manual_seed(N + K)
    x = torch.randn(B * T, C, device=gpu).to(torch.bfloat16)
    wp = (0.3 * torch.randn(N, K, C, device=gpu)).to(torch.bfloat16)
    b = torch.randn(N, device=gpu)
    a_ = torch.randn(B * T, N, device=gpu).to(torch.bfloat16) if aux else None
    r_ = torch.randn(B * T, N, device=gpu).to(torch.bfloat16) if res else None
    lib = L.lib()
    outs = []
    # (key 3, key 44): the streaming kernel on its 768-row tiles (default), on
    # 256-row (44 = 1) and 1024-row (44 = 2) tiles, then the generic kernel
    for v, t44 in ((0, 0), (0, 1), (0, 2), (1, 0)):
        prev, prev44 = lib.sel_tune(3, v), lib.sel_tune(44, t44)
        try:
            outs.append(CO.prim(d, x, wp, bias=b, aux=a_, res=r_).float())
        finally:
            lib.sel_tune(3, prev)
            lib.sel_tune(44, prev44)
    for o in outs[:3]:
        e = ((o - outs[-1]).norm() / outs[-1].norm()).item()
        assert e < 4e-3, e
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])  # tiling only: same bits


@pytest.mark.parametrize("C,K,dil,pad_mode,elu,bias,out32,T", [
    (32, 7, 1, 0, 0, 0, 1, 24000), (32, 7, 1, 0, 0, 0, 0, 1000), (64, 7, 3, 0, 1, 1, 1, 777),
    (64, 3, 1, 1, 0, 1, 0, 500), (32, 2, 1, 1, 1, 0, 1, 61), (32, 7, 9, 0, 0, 1, 0, 40)])
def test_one_output_channel_conv(gpu, C, K, dil, pad_mode, elu, bias, out32, T):
    """N = 1 convs (the decoder's last layer, whose fp32 output feeds the
    losses: decoder.conv2.out_float) in bf16 and fp32 output against fp64 of
    the same bf16 operands: ragged T and T < halo, zero and replicate padding.
    (A dedicated one-output-channel kernel was measured slower than the tiled
    kernel in round 6 -- 87-92 against 37 us -- and dropped.)"""
    from sel import convops as CO
    B = 3
    pad = (K - 1) * dil if pad_mode == 0 else 1
    d = CO.ConvDesc(B * T, T, C, 1, K, dil, pad, CO.PAD_ZERO if pad_mode == 0 else CO.PAD_REPLICATE, elu,
                    1 if bias else 0)
    torch.manual_seed(C + K + T)
    x = torch.randn(B * T, C, device=gpu).to(torch.bfloat16)
    wp = (0.3 * torch.randn(1, K, C, device=gpu)).to(torch.bfloat16)
    b = torch.randn(1, device=gpu) if bias else None
    od = torch.float32 if out32 else torch.bfloat16
    o = CO.prim(d, x, wp, bias=b, out_dtype=od).double()
    # fp64 truth of the same operands (the ELU'd input rounded to bf16 as the kernels stage it)
    xt = x.double().view(B, T, C)
    if elu:
        xt = torch.nn.functional.elu(xt).to(torch.bfloat16).double()
    xp = torch.nn.functional.pad(xt.transpose(1, 2), (pad, (K - 1) * dil - pad),
                                 mode="constant" if pad_mode == 0 else "replicate")
    ref = torch.nn.functional.conv1d(xp, wp.double().permute(0, 2, 1), dilation=dil).transpose(1, 2).reshape(-1, 1)
    if bias:
        ref = ref + b.double()
    e = ((o - ref).norm() / ref.norm()).item()
    assert e < (1e-5 if out32 else 4e-3), e


# (C, N, K, dil, pad_mode, in_elu, aux, res, bias, B, T): every thin-kernel instance in
# its forward and adjoint forms, plus ragged T (tails shorter than one tile) and T < halo
THIN_SHAPES = [(32, 32, 7, 9, 0, 1, 0, 0, 0, 3, 1000), (32, 32, 7, 9, 0, 0, 1, 1, 0, 2, 777),
               (32, 32, 1, 1, 0, 1, 0, 1, 0, 3, 1000), (32, 32, 1, 1, 0, 0, 1, 0, 0, 2, 300),
               (64, 64, 7, 3, 0, 1, 0, 0, 0, 3, 800), (64, 64, 7, 1, 0, 0, 1, 1, 0, 2, 130),
               (64, 64, 1, 1, 0, 1, 0, 1, 0, 3, 800), (96, 64, 3, 1, 0, 0, 0, 0, 64, 4, 333),
               (96, 64, 2, 1, 0, 0, 0, 0, 0, 2, 500), (32, 32, 7, 9, 0, 1, 0, 0, 0, 2, 40),
               (128, 128, 1, 1, 0, 1, 0, 1, 0, 3, 1000), (128, 128, 1, 1, 0, 0, 1, 0, 0, 2, 333),
               (64, 96, 2, 1, 1, 0, 0, 0, 96, 3, 1000), (64, 96, 3, 1, 0, 0, 0, 0, 0, 2, 777),
               (64, 96, 2, 1, 1, 0, 0, 0, 96, 2, 61)]


@pytest.mark.parametrize("shape", THIN_SHAPES, ids=lambda s: "C{}N{}K{}d{}e{}a{}r{}T{}".format(*s[:3], s[3], *s[5:8],
                                                                                               s[10]))
def test_thin_kernel_matches_tiled(gpu, shape):
    """The weight-stationary thin kernel (tune key 4 = 0) against the tiled kernel
    (key 4 = 1) on the same bf16 operands, causal (pad (K-1)*dil) and adjoint
    (pad 0) forms: both accumulate in fp32 (different order) and round once to
    bf16 -> within one bf16 ulp (4e-3 norm-wise), and against an fp64 reference
    of the same bf16 operands within bf16 output rounding (4e-3)."""
    from sel import _lib as L
    from sel import convops as CO
    C, N, K, dil, mode, elu, aux, res, bias, B, T = shape
    torch.manual_seed(C + N + K + T)
    lib = L.lib()
    prev42 = lib.sel_tune(42, 1)  # the 128-channel 1x1 on the thin kernel (k_pw_bf16 off)
    try:
        _thin_vs_tiled(lib, CO, C, N, K, dil, mode, elu, aux, res, bias, B, T, gpu)
    finally:
        lib.sel_tune(42, prev42)


def _thin_vs_tiled(lib, CO, C, N, K, dil, mode, elu, aux, res, bias, B, T, gpu):
    for pad in ((K - 1) * dil, 0):
        d = CO.ConvDesc(B * T, T, C, N, K, dil, pad, mode, elu, bias)
        x = torch.randn(B * T, C, device=gpu).to(torch.bfloat16)
        wp = (0.2 * torch.randn(N, K, C, device=gpu)).to(torch.bfloat16)
        b = torch.randn(bias, device=gpu) if bias else None
        a_ = torch.randn(B * T, N, device=gpu).to(torch.bfloat16) if aux else None
        r_ = torch.randn(B * T, N, device=gpu).to(torch.bfloat16) if res else None
        assert CO.fwd_kernel_name(d, torch.bfloat16, torch.bfloat16).startswith("k_conv_thin_bf16")
        outs = []
        for v in (0, 1):
            prev = lib.sel_tune(4, v)
            try:
                outs.append(CO.prim(d, x, wp, bias=b, aux=a_, res=r_).double())
            finally:
                lib.sel_tune(4, prev)
        e = ((outs[0] - outs[1]).norm() / outs[1].norm()).item()
        assert e < 4e-3, (pad, e)
        # fp64 reference of the same bf16 operands
        xa = x.double().view(B, T, C)
        if elu:
            xa = torch.where(xa > 0, xa, torch.expm1(xa)).to(torch.bfloat16).double()
        ref = torch.zeros(B, T, N, dtype=torch.float64, device=gpu)
        for k in range(K):
            idx = torch.arange(T, device=gpu) + k * dil - pad
            if mode == CO.PAD_REPLICATE:
                xs = xa[:, idx.clamp(0, T - 1)]
            else:
                ok = (idx >= 0) & (idx < T)
                xs = torch.zeros(B, T, C, dtype=torch.float64, device=gpu)
                xs[:, ok] = xa[:, idx[ok]]
            ref += torch.einsum("btc,nc->btn", xs, wp[:, k, :].double())
        ref = ref.view(B * T, N)
        if bias:
            ref += b.double().repeat(N // bias)
        if aux:
            ref *= torch.where(a_.double() > 0, 1.0, torch.exp(a_.double()))
        if res:
            ref += r_.double()
        e = ((outs[0] - ref).norm() / ref.norm()).item()
        assert e < 4e-3, (pad, e)


# (C, rows, T, in_elu, aux, res, bias): the RU256 1x1 forward (ELU'd h, residual x)
# and dgrad (ELU'(h) epilogue) at C3 size, ragged row counts (tails of a block's
# range and of a 32-row sub-tile), fewer rows than one sub-tile, bias, both
# epilogue operands, and the 128-wide instance (tune key 42 = 2)
PW_SHAPES = [(256, 25600, 400, 1, 0, 1, 0), (256, 25600, 400, 0, 1, 0, 0), (256, 6393, 6393, 1, 1, 1, 256),
             (256, 5, 5, 0, 0, 0, 0), (256, 1000, 200, 0, 0, 1, 256), (256, 70001, 70001, 1, 0, 1, 0),
             (128, 128000, 2000, 1, 0, 1, 0), (128, 777, 777, 0, 1, 0, 0)]


@pytest.mark.parametrize("shape", PW_SHAPES, ids=lambda s: "C{}r{}e{}a{}r{}b{}".format(s[0], s[1], *s[3:]))
def test_pointwise_kernel_matches_tiled(gpu, shape):
    """k_pw_bf16 (weight-stationary 1x1, tune key 42) against the kernels it
    replaces (key 42 = 1; k_conv_fwd_bf16<64, 128, 1, 1> at 256 channels, the
    thin kernel at 128): the same 32x32x16 MFMA chain in the same channel
    order and the same epilogue roundings -> bit-identical (the RU forms: one
    epilogue operand);
    against fp64 of the same bf16 operands within bf16 output rounding."""
    from sel import _lib as L
    from sel import convops as CO
    C, rows, T, elu, aux, res, bias = shape
    torch.manual_seed(C + rows)
    lib = L.lib()
    d = CO.ConvDesc(rows, T, C, C, 1, 1, 0, 0, elu, bias)
    x = torch.randn(rows, C, device=gpu).to(torch.bfloat16)
    wp = (0.1 * torch.randn(C, 1, C, device=gpu)).to(torch.bfloat16)
    b = torch.randn(bias, device=gpu) if bias else None
    a_ = torch.randn(rows, C, device=gpu).to(torch.bfloat16) if aux else None
    r_ = torch.randn(rows, C, device=gpu).to(torch.bfloat16) if res else None
    outs = []
    for v in (2, 1):
        prev = lib.sel_tune(42, v)
        try:
            name = CO.fwd_kernel_name(d, torch.bfloat16, torch.bfloat16, bool(aux or res))
            assert name.startswith("k_pw_bf16") == (v == 2), name
            outs.append(CO.prim(d, x, wp, bias=b, aux=a_, res=r_))
        finally:
            lib.sel_tune(42, prev)
    if not (aux and res):
        assert torch.equal(outs[0], outs[1])
    else:  # with both epilogue operands the tiled kernel's ELU'(aux) * v + res may be contracted to an FMA
        e = ((outs[0].double() - outs[1].double()).norm() / outs[1].double().norm()).item()
        assert e < 4e-3, e
    xa = x.double()
    if elu:
        xa = torch.where(xa > 0, xa, torch.expm1(xa)).to(torch.bfloat16).double()
    ref = xa @ wp[:, 0, :].double().t()
    if bias:
        ref += b.double()
    if aux:
        ref *= torch.where(a_.double() > 0, 1.0, torch.exp(a_.double()))
    if res:
        ref += r_.double()
    e = ((outs[0].double() - ref).norm() / ref.norm()).item()
    assert e < 4e-3, e


@pytest.mark.parametrize("epi", [0, 1, 2, 3])
@pytest.mark.parametrize("shape", [(32, 32, 7, 9, 0, 1, 0, 0, 0, 3, 1000), (32, 32, 7, 9, 0, 0, 1, 1, 0, 2, 777),
                                   (32, 32, 7, 1, 0, 0, 1, 0, 0, 5, 600), (64, 64, 7, 3, 0, 0, 1, 1, 0, 3, 800),
                                   (64, 64, 7, 1, 0, 0, 1, 0, 0, 2, 333)],
                         ids=lambda s: "C{}N{}K{}d{}a{}r{}T{}".format(*s[:4], s[6], s[7], s[10]))
def test_thin_kernel_multi_tile_loops(gpu, shape, epi):
    """Many tiles per workgroup (tune key 5 = 3 workgroups): the thin kernel's
    tile loop with and without the epilogue-operand prefetch and the split
    (two-barrier) loop (tune key 11 bits), across batch boundaries and ragged
    tails, equals the single-tile-per-workgroup launch bit for bit (same
    per-tile arithmetic, only the schedule differs)."""
    from sel import _lib as L
    from sel import convops as CO
    C, N, K, dil, mode, elu, aux, res, bias, B, T = shape
    torch.manual_seed(T + epi)
    lib = L.lib()
    for pad in ((K - 1) * dil, 0):
        d = CO.ConvDesc(B * T, T, C, N, K, dil, pad, mode, elu, bias)
        x = torch.randn(B * T, C, device=gpu).to(torch.bfloat16)
        wp = (0.2 * torch.randn(N, K, C, device=gpu)).to(torch.bfloat16)
        a_ = torch.randn(B * T, N, device=gpu).to(torch.bfloat16) if aux else None
        r_ = torch.randn(B * T, N, device=gpu).to(torch.bfloat16) if res else None
        assert CO.fwd_kernel_name(d, torch.bfloat16, torch.bfloat16).startswith("k_conv_thin_bf16")
        ref = CO.prim(d, x, wp, aux=a_, res=r_).clone()
        p5, p11 = lib.sel_tune(5, 3), lib.sel_tune(11, epi)
        try:
            got = CO.prim(d, x, wp, aux=a_, res=r_).clone()
        finally:
            lib.sel_tune(5, p5)
            lib.sel_tune(11, p11)
        assert torch.equal(got, ref), (pad, (got.float() - ref.float()).abs().max().item())


# (C, dil, bias, B, T): the fused residual-unit forward's instances at the
# AudioDec dilations, ragged tails (T not a multiple of the tile rows) and T < halo
RU_SHAPES = [(32, 1, 0, 2, 1000), (32, 3, 0, 3, 777), (32, 9, 1, 2, 1000), (32, 9, 0, 2, 40),
             (32, 9, 1, 64, 24000),   # the C3 size (k_ru32_fwd4 under key 70 too)
             (64, 1, 0, 2, 500), (64, 3, 1, 3, 333), (64, 9, 0, 2, 260), (64, 9, 1, 2, 40),
             (64, 9, 1, 8, 8000),
             # 128 channels: k_conv_wss<7, 16, 128> with the 1x1 in its epilogue (round 6,
             # where conv1 runs on that tile: >= 65536 rows): 250-row tiles, a ragged
             # last tile (T = 1990: 249 + 247), one-tile samples, and the C3 size
             (128, 1, 1, 33, 2000), (128, 3, 0, 34, 1990), (128, 9, 1, 132, 500), (128, 9, 0, 256, 256),
             (128, 3, 1, 64, 2000)]


@pytest.mark.parametrize("shape", RU_SHAPES, ids=lambda s: "C{}d{}b{}B{}T{}".format(*s))
def test_fused_residual_unit_matches_two_calls(gpu, shape, monkeypatch):
    """sel_resunit_fwd (one launch) against the two-primitive path (conv1 with
    ELU prologue, then 1x1 with ELU prologue + residual) on the same bf16
    operands: h and out within one bf16 ulp norm-wise (4e-3), and against an
    fp64 reference of the same operands within bf16 rounding (1e-2)."""
    from sel import convops as CO
    C, dil, bias, B, T = shape
    torch.manual_seed(C + dil + T)
    x = (0.5 * torch.randn(B * T, C, device=gpu)).to(torch.bfloat16)
    w1 = 0.1 * torch.randn(C, C, 7, device=gpu)
    w2 = 0.2 * torch.randn(C, C, 1, device=gpu)
    b1 = torch.randn(C, device=gpu) if bias else None
    b2 = torch.randn(C, device=gpu) if bias else None
    d1 = CO.ConvDesc(B * T, T, C, C, 7, dil, 6 * dil, CO.PAD_ZERO, 1, C if bias else 0)
    d2 = CO.ConvDesc(B * T, T, C, C, 1, 1, 0, CO.PAD_ZERO, 1, C if bias else 0)
    wp1 = CO.pack(CO.PACK_FWD, w1, 1, torch.bfloat16)
    wp2 = CO.pack(CO.PACK_FWD, w2, 1, torch.bfloat16)
    if C == 128:
        assert CO.ru128_fused_ok(d1, torch.bfloat16)
        from sel import _lib as Lb
        p69 = Lb.lib().sel_tune(69, 1)   # off: the two-launch path
        try:
            assert not CO.ru128_fused_ok(d1, torch.bfloat16)
        finally:
            Lb.lib().sel_tune(69, p69)
    else:
        assert CO.ru_fused_ok(d1, torch.bfloat16)
    h, out = CO.resunit_fwd(d1, x, wp1, b1, wp2, b2)
    h_ref = CO.prim(d1, x, wp1, bias=b1)
    out_ref = CO.prim(d2, h_ref, wp2, bias=b2, res=x)
    # k_ru32_fwd / k_ru64_fwd / k_conv_wss RU: same MFMA order and rounding points as the two calls
    assert torch.equal(h, h_ref), (h.float() - h_ref.float()).abs().max().item()
    assert torch.equal(out, out_ref), (out.float() - out_ref.float()).abs().max().item()
    if C == 32:
        # k_ru32_fwd4 (tune key 70 = 1: W1 in LDS, swizzled ELU(x) rows, residual
        # re-read from global memory): the same operands and MFMA order, same bits
        from sel import _lib as Lb
        p70 = Lb.lib().sel_tune(70, 1)
        try:
            h4, out4 = CO.resunit_fwd(d1, x, wp1, b1, wp2, b2)
        finally:
            Lb.lib().sel_tune(70, p70)
        assert torch.equal(h4, h_ref), (h4.float() - h_ref.float()).abs().max().item()
        assert torch.equal(out4, out_ref), (out4.float() - out_ref.float()).abs().max().item()
    if C == 64:
        # the round-2 LDS-staged instance (tune key 24 = -1): within one bf16 ulp norm-wise
        from sel import _lib as Lb
        lib = Lb.lib()
        p24 = lib.sel_tune(24, -1)
        try:
            h2, out2 = CO.resunit_fwd(d1, x, wp1, b1, wp2, b2)
        finally:
            lib.sel_tune(24, p24)
        for a_, b_ in ((h2, h_ref), (out2, out_ref)):
            e = ((a_.float() - b_.float()).norm() / b_.float().norm()).item()
            assert e < 4e-3, e
    # fp64 reference of the same bf16 operands
    elu = lambda v: torch.where(v > 0, v, torch.expm1(v))
    xa = elu(x.double()).to(torch.bfloat16).double().view(B, T, C)
    w1q = wp1.double().view(C, 7, C)
    hr = torch.zeros(B, T, C, dtype=torch.float64, device=gpu)
    for k in range(7):
        idx = torch.arange(T, device=gpu) + k * dil - 6 * dil
        ok = idx >= 0
        xs = torch.zeros(B, T, C, dtype=torch.float64, device=gpu)
        xs[:, ok] = xa[:, idx[ok]]
        hr += torch.einsum("btc,nc->btn", xs, w1q[:, k, :])
    if bias:
        hr += b1.double()
    ha = elu(hr.to(torch.bfloat16).double()).to(torch.bfloat16).double()
    outr = x.double().view(B, T, C) + torch.einsum("btc,nc->btn", ha, wp2.double().view(C, C))
    if bias:
        outr += b2.double()
    for a_, b_ in ((h, hr), (out, outr)):
        e = ((a_.double().view(B, T, C) - b_).norm() / b_.norm()).item()
        assert e < 1e-2, e


RU32_BWD_SHAPES = [(32, 1, 0, 2, 1000), (32, 3, 1, 3, 777), (32, 9, 1, 2, 1000), (32, 9, 0, 2, 40),
                   (32, 9, 1, 4, 24000), (64, 1, 0, 2, 500), (64, 3, 1, 3, 333), (64, 9, 0, 2, 40),
                   (64, 9, 1, 8, 8000)]


@pytest.mark.parametrize("shape", RU32_BWD_SHAPES, ids=lambda s: "C{}d{}b{}B{}T{}".format(*s))
def test_resunit32_bwd_matches_two_calls(gpu, shape):
    """sel_resunit_bwd (one launch, k_ru32_bwd / k_ru64_bwd) against the two
    adjoint primitive calls of ResidualUnitFn's unfused backward on the same
    bf16 operands: gh bit-identical, gx within one bf16 ulp on < 0.1% of the
    elements (same MFMA order, same rounding points), ragged tails, T < halo and
    the C3 sizes (T = 24000 at 32 channels, 8000 at 64)."""
    from sel import convops as CO
    C, dil, bias, B, T = shape
    torch.manual_seed(dil + T)
    x = (0.5 * torch.randn(B * T, C, device=gpu)).to(torch.bfloat16)
    h = (0.5 * torch.randn(B * T, C, device=gpu)).to(torch.bfloat16)
    g = (0.5 * torch.randn(B * T, C, device=gpu)).to(torch.bfloat16)
    w1 = 0.1 * torch.randn(C, C, 7, device=gpu)
    w2 = 0.2 * torch.randn(C, C, 1, device=gpu)
    d1 = CO.ConvDesc(B * T, T, C, C, 7, dil, 6 * dil, CO.PAD_ZERO, 1, C if bias else 0)
    d2 = CO.ConvDesc(B * T, T, C, C, 1, 1, 0, CO.PAD_ZERO, 1, C if bias else 0)
    wp1, wd1 = CO.PACKS.get(CO.PACK_FWD, w1, 1, torch.bfloat16)
    wp2, wd2 = CO.PACKS.get(CO.PACK_FWD, w2, 1, torch.bfloat16)
    assert CO.ru_bwd_fused_ok(d1, torch.bfloat16)
    gx, gh = CO.resunit_bwd(d1, g, h, x, wd1, wd2, True)
    gh_ref = CO.prim(d2.adjoint(), g, wd2, aux=h)
    gx_ref = CO.prim(d1.adjoint(), gh_ref, wd1, aux=x, res=g)
    assert torch.equal(gh, gh_ref), ((gh.float() - gh_ref.float()).abs().max().item())
    _ulp_close(gx, gx_ref)
    gx2, gh2 = CO.resunit_bwd(d1, g, h, x, wd1, wd2, False)
    assert gh2 is None and torch.equal(gx2, gx)


RU32_WGRAD_SHAPES = [(1, 1, 2, 1000), (3, 1, 3, 777), (9, 0, 2, 40), (9, 1, 1, 130), (9, 1, 64, 24000),
                     (3, 1, 64, 24000)]


@pytest.mark.parametrize("shape", RU32_WGRAD_SHAPES, ids=lambda s: "d{}b{}B{}T{}".format(*s))
def test_resunit32_bwd_wgrad_fused(gpu, shape):
    """sel_resunit_bwd_wgrad (k_ru32_bwdw: gx AND both weight gradients in one
    launch, per-block partials reduced by sel_wgrad_finish_many) against the
    unfused path on the same bf16 operands: gx bit-identical to k_ru32_bwd (same
    phases), the four weight / bias gradients against the two-launch wgrad
    (another fp32 row-summation order: <= 1e-5 norm-wise) and against fp64 of
    the same bf16 operands (<= 1e-5).  Ragged tails, T < halo, one tile, empty
    blocks (few tiles) and the C3 size (B = 64 x 24000)."""
    from sel import convops as CO
    dil, bias, B, T = shape
    C = 32
    torch.manual_seed(dil + T + B)
    x = (0.5 * torch.randn(B * T, C, device=gpu)).to(torch.bfloat16)
    h = (0.5 * torch.randn(B * T, C, device=gpu)).to(torch.bfloat16)
    g = (0.5 * torch.randn(B * T, C, device=gpu)).to(torch.bfloat16)
    w1 = 0.1 * torch.randn(C, C, 7, device=gpu)
    w2 = 0.2 * torch.randn(C, C, 1, device=gpu)
    d1 = CO.ConvDesc(B * T, T, C, C, 7, dil, 6 * dil, CO.PAD_ZERO, 1, C if bias else 0)
    d2 = CO.ConvDesc(B * T, T, C, C, 1, 1, 0, CO.PAD_ZERO, 1, C if bias else 0)
    wp1, wd1 = CO.PACKS.get(CO.PACK_FWD, w1, 1, torch.bfloat16)
    wp2, wd2 = CO.PACKS.get(CO.PACK_FWD, w2, 1, torch.bfloat16)
    gx, gw1, gb1, gw2, gb2 = CO.resunit_bwd_wgrad(d1, g, h, x, wd1, wd2, (C, C, 7), (C, C, 1), bool(bias),
                                                  bool(bias), None, None)
    gx_ref, gh_ref = CO.resunit_bwd(d1, g, h, x, wd1, wd2, True)
    assert torch.equal(gx, gx_ref), (gx.float() - gx_ref.float()).abs().max().item()
    gw2_ref, gb2_ref = CO.wgrad_torch(d2, g, h, CO.PACK_FWD, (C, C, 1), 1, bool(bias))
    gw1_ref, gb1_ref = CO.wgrad_torch(d1, gh_ref, x, CO.PACK_FWD, (C, C, 7), 1, bool(bias))
    torch.cuda.synchronize()
    rel = lambda a, b: ((a.double() - b.double()).norm() / b.double().norm()).item()  # noqa: E731
    for name, a_, b_ in (("gw1", gw1, gw1_ref), ("gw2", gw2, gw2_ref)) + \
            ((("gb1", gb1, gb1_ref), ("gb2", gb2, gb2_ref)) if bias else ()):
        assert rel(a_, b_) <= 1e-5, (name, rel(a_, b_))
    # fp64 of the same bf16 operands: gW1[n,c,k] = sum_t gh[t,n] ELU(x)[t + (k-6) dil, c]
    elu = lambda v: torch.where(v > 0, v, torch.expm1(v)).to(torch.bfloat16).double()  # noqa: E731
    ghd = gh_ref.double().view(B, T, C)
    xe = elu(x.double()).view(B, T, C)
    ref1 = torch.zeros(C, C, 7, dtype=torch.float64, device=gpu)
    for k in range(7):
        s = (6 - k) * dil
        if s < T:
            ref1[:, :, k] = torch.einsum("btn,btc->nc", ghd[:, s:], xe[:, :T - s])
    ref2 = torch.einsum("tn,tc->nc", g.double(), elu(h.double()))[:, :, None]
    assert rel(gw1, ref1) <= 1e-5, rel(gw1, ref1)
    assert rel(gw2, ref2) <= 1e-5, rel(gw2, ref2)
    if bias:
        assert rel(gb1, ghd.sum((0, 1))) <= 1e-5 and rel(gb2, g.double().sum(0)) <= 1e-5


RU64_WGRAD_SHAPES = [(1, 1, 2, 500), (3, 1, 3, 333), (9, 0, 2, 40), (9, 1, 1, 130), (9, 1, 8, 8000),
                     (1, 0, 64, 8000), (3, 1, 64, 8000), (9, 1, 64, 8000)]


@pytest.mark.parametrize("shape", RU64_WGRAD_SHAPES, ids=lambda s: "d{}b{}B{}T{}".format(*s))
def test_resunit64_bwd_wgrad_fused(gpu, shape):
    """sel_resunit_bwd_wgrad at 64 channels (k_ru64_bwdw: eight waves, gx waves
    beside weight-gradient waves, per-block partials reduced by
    sel_wgrad_finish_many) against the unfused path on the same bf16 operands:
    gx bit-identical to k_ru64_bwd (same gx phase), the four weight / bias
    gradients against the two k_wgrad3 launches (another fp32 row-summation
    order: <= 1e-5 norm-wise) and against fp64 of the same bf16 operands
    (<= 1e-5).  Ragged tails, T < halo, one tile, empty blocks and the C3 RU64
    size (B = 64 x 8000) at the three dilations."""
    from sel import convops as CO
    dil, bias, B, T = shape
    C = 64
    torch.manual_seed(dil + T + B + 64)
    x = (0.5 * torch.randn(B * T, C, device=gpu)).to(torch.bfloat16)
    h = (0.5 * torch.randn(B * T, C, device=gpu)).to(torch.bfloat16)
    g = (0.5 * torch.randn(B * T, C, device=gpu)).to(torch.bfloat16)
    w1 = 0.1 * torch.randn(C, C, 7, device=gpu)
    w2 = 0.2 * torch.randn(C, C, 1, device=gpu)
    d1 = CO.ConvDesc(B * T, T, C, C, 7, dil, 6 * dil, CO.PAD_ZERO, 1, C if bias else 0)
    d2 = CO.ConvDesc(B * T, T, C, C, 1, 1, 0, CO.PAD_ZERO, 1, C if bias else 0)
    wp1, wd1 = CO.PACKS.get(CO.PACK_FWD, w1, 1, torch.bfloat16)
    wp2, wd2 = CO.PACKS.get(CO.PACK_FWD, w2, 1, torch.bfloat16)
    assert CO.ru_wgrad_fused_ok(d1, torch.bfloat16)
    gx, gw1, gb1, gw2, gb2 = CO.resunit_bwd_wgrad(d1, g, h, x, wd1, wd2, (C, C, 7), (C, C, 1), bool(bias),
                                                  bool(bias), None, None)
    gx_ref, gh_ref = CO.resunit_bwd(d1, g, h, x, wd1, wd2, True)
    assert torch.equal(gx, gx_ref), (gx.float() - gx_ref.float()).abs().max().item()
    gw2_ref, gb2_ref = CO.wgrad_torch(d2, g, h, CO.PACK_FWD, (C, C, 1), 1, bool(bias))
    gw1_ref, gb1_ref = CO.wgrad_torch(d1, gh_ref, x, CO.PACK_FWD, (C, C, 7), 1, bool(bias))
    torch.cuda.synchronize()
    rel = lambda a, b: ((a.double() - b.double()).norm() / b.double().norm()).item()  # noqa: E731
    for name, a_, b_ in (("gw1", gw1, gw1_ref), ("gw2", gw2, gw2_ref)) + \
            ((("gb1", gb1, gb1_ref), ("gb2", gb2, gb2_ref)) if bias else ()):
        assert rel(a_, b_) <= 1e-5, (name, rel(a_, b_))
    elu = lambda v: torch.where(v > 0, v, torch.expm1(v)).to(torch.bfloat16).double()  # noqa: E731
    ghd = gh_ref.double().view(B, T, C)
    xe = elu(x.double()).view(B, T, C)
    ref1 = torch.zeros(C, C, 7, dtype=torch.float64, device=gpu)
    for k in range(7):
        s = (6 - k) * dil
        if s < T:
            ref1[:, :, k] = torch.einsum("btn,btc->nc", ghd[:, s:], xe[:, :T - s])
    ref2 = torch.einsum("tn,tc->nc", g.double(), elu(h.double()))[:, :, None]
    assert rel(gw1, ref1) <= 1e-5, rel(gw1, ref1)
    assert rel(gw2, ref2) <= 1e-5, rel(gw2, ref2)
    if bias:
        assert rel(gb1, ghd.sum((0, 1))) <= 1e-5 and rel(gb2, g.double().sum(0)) <= 1e-5


def _ulp_close(a, b, frac=1e-3):
    """bf16 tensors equal up to one ulp on at most `frac` of the elements: the
    ELU'(x) factor's hardware exp rounds differently in the fused kernel on a
    few ties (measured at T = 24000: 47 of 96000 rows, equally close to fp64)."""
    af, bf = a.double(), b.double()
    m = torch.maximum(af.abs(), bf.abs())
    _, ex = torch.frexp(m)
    ulp = torch.ldexp(torch.ones_like(m), ex - 8)  # bf16: 8 significant bits
    d = (af - bf).abs()
    tiny = 1e-6 * bf.abs().max()
    assert bool((d <= ulp + tiny).all()), float((d - ulp).max())
    assert float((d > 0).float().mean()) <= frac, float((d > 0).float().mean())


@pytest.mark.parametrize("C", [32, 64, 128])
def test_resunit32_autograd_fused_vs_unfused(gpu, monkeypatch, C):
    """ResidualUnitFn at 32 / 64 / 128 channels: forward and all five gradients
    with the fused launches (default; at 128 the forward only, k_conv_wss RU)
    equal the unfused primitive path (SEL_RU_FUSED=0)."""
    from sel import convops as CO
    torch.manual_seed(5)
    B, T, dil = (2, 3000, 3) if C < 128 else (24, 3000, 3)   # 128: >= 65536 rows (the fused tile's range)
    x0 = (0.5 * torch.randn(B, T, C, device=gpu)).to(torch.bfloat16)
    w1 = (0.1 * torch.randn(C, C, 7, device=gpu)).requires_grad_(True)
    b1 = torch.randn(C, device=gpu).requires_grad_(True)
    w2 = (0.2 * torch.randn(C, C, 1, device=gpu)).requires_grad_(True)
    b2 = torch.randn(C, device=gpu).requires_grad_(True)
    gy = (0.5 * torch.randn(B, T, C, device=gpu)).to(torch.bfloat16)
    res = {}
    for mode in ("", "0"):
        monkeypatch.setattr(CO, "RU_FUSED", mode)
        x = x0.clone().requires_grad_(True)
        for p_ in (w1, b1, w2, b2):
            p_.grad = None
        y = CO.ResidualUnitFn.apply(x, w1, b1, w2, b2, dil)
        y.backward(gy)
        res[mode] = [y.detach().clone(), x.grad.clone()] + [p_.grad.clone() for p_ in (w1, b1, w2, b2)]
    assert torch.equal(res[""][0], res["0"][0])  # forward: bit-identical
    _ulp_close(res[""][1], res["0"][1])          # gx
    for a_, b_ in zip(res[""][2:], res["0"][2:]):  # weight / bias grads (fp32) through the same gh
        assert ((a_ - b_).norm() / b_.norm()).item() < 1e-3


def test_deferred_wgrad_reduction_bit_identical(gpu, monkeypatch):
    """Batched weight-gradient reductions (sel_conv_wgrad_partials + one
    sel_wgrad_finish_many launch from the autograd final callback) give the
    same bits as the per-layer reduction passes, for a residual unit (fused
    bwd path: k7 + 1x1, with biases), a strided conv, a transposed conv and a
    single-channel first conv; with a pre-existing .grad (accumulation) the
    layer is not deferred and the sum is still exact."""
    from sel import convops as CO
    torch.manual_seed(11)
    B, T = 2, 3000

    def run(defer, accumulate=False):
        monkeypatch.setattr(CO, "WGRAD_DEFER", defer)
        g = torch.Generator(device=gpu).manual_seed(3)
        x0 = (0.5 * torch.randn(B, T, 1, device=gpu, generator=g)).to(torch.bfloat16)
        w0 = (0.3 * torch.randn(32, 1, 7, device=gpu, generator=g)).requires_grad_(True)
        w1 = (0.1 * torch.randn(32, 32, 7, device=gpu, generator=g)).requires_grad_(True)
        b1 = torch.randn(32, device=gpu, generator=g).requires_grad_(True)
        w2 = (0.2 * torch.randn(32, 32, 1, device=gpu, generator=g)).requires_grad_(True)
        b2 = torch.randn(32, device=gpu, generator=g).requires_grad_(True)
        ws = (0.1 * torch.randn(64, 32, 6, device=gpu, generator=g)).requires_grad_(True)
        bs = torch.randn(64, device=gpu, generator=g).requires_grad_(True)
        wt = (0.1 * torch.randn(64, 32, 6, device=gpu, generator=g)).requires_grad_(True)
        bt = torch.randn(32, device=gpu, generator=g).requires_grad_(True)
        params = (w0, w1, b1, w2, b2, ws, bs, wt, bt)
        if accumulate:
            for p_ in params:
                p_.grad = torch.ones_like(p_)
        h = CO.ConvLayerFn.apply(x0, w0, None, CO.PACK_FWD, 1, 1)
        h = CO.ResidualUnitFn.apply(h, w1, b1, w2, b2, 3)
        h = CO.ConvLayerFn.apply(h, ws, bs, CO.PACK_FWD, 3, 1)
        y = CO.ConvLayerFn.apply(h, wt, bt, CO.PACK_CONVT, 3, 1)
        y.float().square().mean().backward()
        torch.cuda.synchronize()
        return [p_.grad.clone() for p_ in params]

    ref = run(False)
    got = run(True)
    assert not CO._DEFERRED
    for i, (a_, b_) in enumerate(zip(got, ref)):
        assert torch.equal(a_, b_), (i, (a_ - b_).abs().max().item())
    acc = run(True, accumulate=True)
    for a_, b_ in zip(acc, ref):
        assert torch.equal(a_, b_ + 1.0)
    # tune key 68 = 1: the batched finish sums partial split groups four loads
    # at a time (the pre-round-6 order): the same sums to fp32 rounding
    from sel import _lib as L
    prev = L.lib().sel_tune(68, 1)
    try:
        four = run(True)
    finally:
        L.lib().sel_tune(68, prev)
    for i, (a_, b_) in enumerate(zip(four, ref)):
        assert torch.allclose(a_, b_, rtol=1e-5, atol=1e-6 * b_.abs().max().item()), i


@pytest.mark.parametrize("per_element", [0, 1])
def test_pack_many_matches_per_layer_pack(gpu, per_element):
    """PackCache's one-launch refresh (sel_pack_many_host: the tiled
    k_pack_tiles, or the per-element k_pack_many_arg under tune key 60 = 1)
    writes the same bytes as sel_pack_weight + sel_pack_dgrad per layer, for
    the three packed kinds (causal conv, phase-view strided conv, transposed
    conv; ragged 32-tiles included) in both dtypes."""
    from sel import _lib as Lb
    from sel import convops as CO
    prev = Lb.lib().sel_tune(60, per_element)
    try:
        layers = [(CO.PACK_FWD, (64, 32, 7), 1), (CO.PACK_FWD, (256, 256, 1), 1),
                  (CO.PACK_FWD_STRIDED, (128, 64, 4), 2), (CO.PACK_FWD_STRIDED, (512, 256, 10), 5),
                  (CO.PACK_CONVT, (256, 128, 6), 3), (CO.PACK_CONVT, (64, 96, 2), 1), (CO.PACK_FWD, (1, 32, 7), 1),
                  (CO.PACK_FWD, (32, 1, 7), 1), (CO.PACK_FWD, (48, 40, 3), 1),
                  (CO.PACK_FWD_STRIDED, (64, 32, 6), 3), (CO.PACK_CONVT, (64, 32, 6), 3)]
        _pack_many_check(gpu, CO, layers)   # 640 + tiles in one launch
        # < 512 tiles (as the small launches of a C3 step)
        _pack_many_check(gpu, CO, [l for l in layers if l[1] != (512, 256, 10)])
    finally:
        Lb.lib().sel_tune(60, prev)


def _pack_many_check(gpu, CO, layers):
    torch.manual_seed(11)
    for dt in (torch.bfloat16, torch.float32):
        cache = CO.PackCache()
        ws = [torch.randn(*shp, device=gpu) for _, shp, _ in layers]
        for (kind, _, stride), w in zip(layers, ws):
            cache.get(kind, w, stride, dt)  # registers the entry
        with torch.no_grad():
            for w in ws:
                w.mul_(1.5)  # every entry stale: the next get refreshes all of them in one launch
        for (kind, _, stride), w in zip(layers, ws):
            wp, wd = cache.get(kind, w, stride, dt)
            ref = CO.pack(kind, w, stride, dt)
            assert torch.equal(wp, ref), (kind, tuple(w.shape), dt)
            assert torch.equal(wd.contiguous(), CO.pack_dgrad(ref)), (kind, tuple(w.shape), dt)
