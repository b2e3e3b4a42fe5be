"""Kernel variants of the discriminator path agree with each other (round-2
kernels; the default path of each shape is checked against fp64 torch in
test_gpu_gan.py):

* k_dconv_pf tiles (tune key 19: 128x64 / 64x64 by size, 256x64, 128x128,
  256x128) run the same MFMA order, so every tile gives the same bits;
* the LDS-staged short-reduction kernels (tune key 18: 1 = the unstaged ones):
  the forward is bit-identical, the weight gradient sums rows in another order;
* the GAN loss terms' 16-B vector path (contiguous last dim, multiple of 8) and
  the per-element path, both against fp64 torch.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

# (tag, cin, cout, Kt, stride, pad, groups, Bs, T): one-group layers of C5 (48 kHz)
PF_LAYERS = [
    ("mpd1_s3", 32, 128, 5, 3, 2, 1, 6, 2001),
    ("mpd2_s3", 128, 512, 5, 3, 2, 1, 6, 667),
    ("mpd4_s1", 1024, 1024, 5, 1, 2, 1, 6, 25),
    ("msd6_k5", 1024, 1024, 5, 1, 2, 1, 2, 48),
]
SHORT_LAYERS = [
    ("msd0_k15", 1, 128, 15, 1, 7, 1, 2, 3000),
    ("mpd0_s3", 1, 32, 5, 3, 2, 1, 6, 6001),
]


def _setup(gpu, shape, dt):
    from sel import dconvops as DC
    tag, cin, cout, Kt, s, pad, G, Bs, T = shape
    sp = DC.LayerSpec(cin, cout, Kt, s, pad, G, True)
    torch.manual_seed(Kt * 13 + cout)
    T_out = sp.t_out(T)
    Ta = DC._roundup(T, s)
    x = torch.zeros(Bs, Ta, cin, device=gpu)
    x[:, :T] = torch.randn(Bs, T, cin, device=gpu)
    w = torch.randn(cout, cin // G, Kt, device=gpu) / (cin // G * Kt) ** 0.5
    b = torch.randn(cout, device=gpu)
    g = torch.randn(Bs, T_out, cout, device=gpu).to(dt).contiguous()
    return sp, x.to(dt), w, b, g, (Bs, T, Ta, T_out)


def _run(sp, x, w, b, g, geo, dt, want_wgrad=False):
    from sel import dconvops as DC
    Bs, T, Ta, T_out = geo
    d = DC._fwd_desc(sp, Bs, T, Ta, T_out, T_out, 0.1)
    y = torch.empty(Bs, T_out, sp.cout, dtype=dt, device=x.device)
    DC.prim(d, x, DC.pack(sp, w, None, dt, 0), y, bias=b)
    db = DC._dgrad_desc(sp, Bs, Ta, T_out, T_out, 0.1, False)
    gin = torch.empty(Bs, Ta, sp.cin, dtype=dt, device=x.device)
    DC.prim(db, g, DC.pack(sp, w, None, dt, 1), gin)
    out = [y, gin]
    if want_wgrad:
        gw, _, gb = DC.wgrad(sp, d, g, x, w, None, True, True)
        out += [gw, gb]
    torch.cuda.synchronize()
    return out


@pytest.mark.parametrize("shape", PF_LAYERS, ids=[s[0] for s in PF_LAYERS])
def test_pf_tiles_bit_identical(gpu, shape):
    from sel import _lib as Lb
    lib = Lb.lib()
    dt = torch.bfloat16
    sp, x, w, b, g, geo = _setup(gpu, shape, dt)
    prev = lib.sel_tune(19, 0)
    try:
        ref = _run(sp, x, w, b, g, geo, dt)
        for v in (1, 2, 3):
            lib.sel_tune(19, v)
            got = _run(sp, x, w, b, g, geo, dt)
            for name, r, o in zip(("fwd", "adjoint"), ref, got):
                assert torch.equal(r, o), (shape[0], v, name, float((r.float() - o.float()).abs().max()))
    finally:
        lib.sel_tune(19, prev)


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
@pytest.mark.parametrize("shape", SHORT_LAYERS, ids=[s[0] for s in SHORT_LAYERS])
def test_short_staged_matches_unstaged(gpu, shape, dtype):
    from sel import _lib as Lb
    lib = Lb.lib()
    dt = torch.float32 if dtype == "fp32" else torch.bfloat16
    sp, x, w, b, g, geo = _setup(gpu, shape, dt)
    prev = lib.sel_tune(18, 1)
    try:
        y0, gi0, gw0, gb0 = _run(sp, x, w, b, g, geo, dt, want_wgrad=True)
        lib.sel_tune(18, 0)
        y1, gi1, gw1, gb1 = _run(sp, x, w, b, g, geo, dt, want_wgrad=True)
    finally:
        lib.sel_tune(18, prev)
    assert torch.equal(y0, y1), float((y0.float() - y1.float()).abs().max())
    assert torch.equal(gi0, gi1)  # the adjoint does not take the short path: same kernel
    # fp32 partial sums over the rows in a different order: ~1e-7 relative
    for a, c in ((gw0, gw1), (gb0, gb1)):
        assert ((a - c).norm() / a.norm()).item() <= 1e-5


@pytest.mark.parametrize("C", [64, 60], ids=["vector", "per_element"])
def test_gan_terms_vector_and_scalar(gpu, C):
    """(B, C, T) views of channels-last (B, T, C) feature maps: C % 8 == 0 takes
    the 16-B vector kernels, C = 60 the per-element ones; fp64 torch reference."""
    from sel import dconvops as DC
    torch.manual_seed(C)
    B, T = 3, 517
    for dt, tol in ((torch.float32, 1e-6), (torch.bfloat16, 1e-6)):
        fa = torch.randn(B, T, C, device=gpu).to(dt)
        fb = torch.randn(B, T, C, device=gpu).to(dt)
        a = fa.permute(0, 2, 1).detach().requires_grad_(True)
        bv = fb.permute(0, 2, 1)
        l1 = DC.l1_mean(a, bv)
        ref = (a.double() - bv.double()).abs().mean()
        assert abs(l1.item() - ref.item()) <= tol * max(1.0, abs(ref.item())), (C, dt, l1.item(), ref.item())
        l1.backward()
        gref = torch.sign(a.double() - bv.double()) / a.numel()
        assert ((a.grad.double() - gref).abs().max() <= 1e-2 * gref.abs().max()).item()
        a2 = fa.permute(0, 2, 1).detach().requires_grad_(True)
        m = DC.mse_to(a2, 1.0)
        mref = ((a2.double() - 1.0) ** 2).mean()
        assert abs(m.item() - mref.item()) <= tol * max(1.0, abs(mref.item()))
        m.backward()
        g2 = 2.0 * (a2.double() - 1.0) / a2.numel()
        assert ((a2.grad.double() - g2).norm() / g2.norm()).item() <= (1e-6 if dt == torch.float32 else 1e-2)


# (tag, cin, cout, Kt, stride, pad, groups, Bs, T): MPD layers at sizes that take
# the warp-specialised kernel (rows x width / 128 >= 65536; Bs = clips x period columns)
WS_LAYERS = [
    ("mpd1_s3", 32, 128, 5, 3, 2, 1, 32, 6150),
    ("mpd2_s3", 128, 512, 5, 3, 2, 1, 32, 1602),
    ("mpd3_s3", 512, 1024, 5, 3, 2, 1, 48, 600),
    ("mpd4_s1", 1024, 1024, 5, 1, 2, 1, 48, 200),
]


@pytest.mark.parametrize("shape", WS_LAYERS, ids=[s[0] for s in WS_LAYERS])
def test_ws_tiles_match_fp64_and_pf(gpu, shape):
    """The MPD's wide layers on conv.hip's warp-specialised 256 x 128 kernel
    (dconv_ws_fwd; tune key 21 = 1 keeps them on k_dconv_pf): forward with
    bias + LeakyReLU and 3 zero rows past the computed ones, adjoint with the
    (+ res) * LeakyReLU'(aux) epilogue, both against fp64 torch of the same bf16
    operands (bound 1e-2 norm-wise: output rounding only) and against the pf
    kernel (another fp32 summation order: <= 5e-3)."""
    from sel import _lib as Lb
    from sel import dconvops as DC
    lib = Lb.lib()
    dt = torch.bfloat16
    tag, cin, cout, Kt, s, pad, G, Bs, T = shape
    sp = DC.LayerSpec(cin, cout, Kt, s, pad, G, True)
    slope = 0.1
    torch.manual_seed(Kt * 31 + cout)
    T_out = sp.t_out(T)
    Ta = DC._roundup(T, s)
    x = torch.zeros(Bs, Ta, cin, device=gpu)
    x[:, :T] = torch.randn(Bs, T, cin, device=gpu)
    x = x.to(dt)
    w = torch.randn(cout, cin, Kt, device=gpu) / (cin * Kt) ** 0.5
    b = torch.randn(cout, device=gpu)
    wq = w.to(dt).double()
    pre = torch.nn.functional.conv1d(x[:, :T].double().permute(0, 2, 1), wq, b.double(), stride=s,
                                     padding=pad).permute(0, 2, 1)
    ref_y = torch.nn.functional.leaky_relu(pre, slope)
    g = torch.randn(Bs, T_out, cout, device=gpu).to(dt)
    aux = torch.randn(Bs, Ta, cin, device=gpu).to(dt)
    res = torch.randn(Bs, Ta, cin, device=gpu).to(dt)
    xr = x[:, :T].double().clone().requires_grad_(True)
    torch.nn.functional.conv1d(xr.permute(0, 2, 1), wq, None, stride=s, padding=pad).permute(0, 2, 1).backward(
        g.double())
    ref_gin = (xr.grad + res[:, :T].double()) * torch.where(aux[:, :T].double() > 0, 1.0, slope)

    def run():
        Tva = T_out + 3
        d = DC._fwd_desc(sp, Bs, T, Ta, T_out, Tva, slope)
        y = torch.full((Bs, Tva, cout), 7.0, dtype=dt, device=gpu)
        DC.prim(d, x, DC.pack(sp, w, None, dt, 0), y, bias=b)
        db = DC._dgrad_desc(sp, Bs, Ta, T_out, T_out, slope, False)
        gin = torch.empty(Bs, Ta, cin, dtype=dt, device=gpu)
        DC.prim(db, g, DC.pack(sp, w, None, dt, 1), gin, aux=aux, res=res)
        torch.cuda.synchronize()
        return y, gin

    prev = lib.sel_tune(21, 0)
    try:
        y, gin = run()
        lib.sel_tune(21, 1)
        y_pf, gin_pf = run()
    finally:
        lib.sel_tune(21, prev)
    assert torch.count_nonzero(y[:, T_out:]).item() == 0
    rel = lambda a, r: ((a.double() - r).norm() / r.norm()).item()  # noqa: E731
    assert rel(y[:, :T_out], ref_y) <= 1e-2, (tag, "fwd", rel(y[:, :T_out], ref_y))
    assert rel(gin[:, :T], ref_gin) <= 1e-2, (tag, "adjoint", rel(gin[:, :T], ref_gin))
    assert rel(y, y_pf.double()) <= 5e-3, (tag, "fwd vs pf", rel(y, y_pf.double()))
    assert rel(gin, gin_pf.double()) <= 5e-3, (tag, "adjoint vs pf", rel(gin, gin_pf.double()))


def test_pack_many_matches_per_layer_pack(gpu):
    """sel_dconv_pack_many (one launch for a chain's stale forms) writes the same
    bytes as one sel_dconv_pack per (layer, mode), with and without weight norm."""
    from sel import dconvops as DC
    torch.manual_seed(7)
    specs = [DC.LayerSpec(1, 32, 5, 3, 2, 1, True), DC.LayerSpec(32, 128, 5, 3, 2, 1, True),
             DC.LayerSpec(128, 128, 41, 2, 20, 4, True), DC.LayerSpec(256, 512, 41, 4, 20, 16, True),
             DC.LayerSpec(1024, 1, 3, 1, 1, 1, False)]
    for dt in (torch.bfloat16, torch.float32):
        for wn in (False, True):
            cache = DC._DPackCache()
            items, ws = [], []
            for sp in specs:
                w = torch.randn(sp.cout, sp.cin // sp.groups, sp.Kt, device=gpu)
                wg = torch.rand(sp.cout, 1, 1, device=gpu) + 0.5 if wn else None
                ws.append((sp, w, wg))
                items += [(sp, w, wg, dt, 0), (sp, w, wg, dt, 1)]
            cache.prefetch(items)
            for sp, w, wg in ws:
                for mode in (0, 1):
                    got = cache.get(sp, w, wg, dt, mode)
                    ref = DC._pack(sp, w, wg, dt, mode)
                    assert torch.equal(got, ref), (sp.cin, sp.cout, sp.Kt, mode, dt, wn)


@pytest.mark.parametrize("shape", [("mpd4_s1", 1024, 1024, 5, 1, 2, 96, 54), ("mpd3_s3", 512, 1024, 5, 3, 2, 96, 162)],
                         ids=["mpd4_s1", "mpd3_s3"])
def test_wgrad_flat_tiles(gpu, shape):
    """k_dwgrad_w3 over the period chain's zero-gapped layout (row pitch P =
    valid rows + 2): flat tiles across sequences (default) vs per-sequence tiles
    (tune key 26 = 1) vs fp64 torch; the gradient's gap rows hold garbage, which
    the row-validity masks must drop."""
    from sel import _lib as Lb
    from sel import dconvops as DC
    lib = Lb.lib()
    tag, cin, cout, Kt, s, pad, Bs, T = shape
    sp = DC.LayerSpec(cin, cout, Kt, s, pad, 1, True)
    torch.manual_seed(cout + T)
    T_out = sp.t_out(T)
    P = T_out + 2                      # output rows per sequence (2 gap rows)
    Ta = P * s                         # input rows per sequence (phase view: P rows)
    x = torch.zeros(Bs, Ta, cin, device=gpu)
    x[:, :T] = torch.randn(Bs, T, cin, device=gpu)
    x = x.to(torch.bfloat16)
    g = torch.randn(Bs, P, cout, device=gpu).to(torch.bfloat16)  # gap rows: garbage
    d = DC._fwd_desc(sp, Bs, T, Ta, T_out, P, 0.1)
    w = torch.randn(cout, cin, Kt, device=gpu)
    prev = lib.sel_tune(26, 0)
    try:
        gw, _, gb = DC.wgrad(sp, d, g, x, w, None, True, True)
        lib.sel_tune(26, 1)
        gw1, _, gb1 = DC.wgrad(sp, d, g, x, w, None, True, True)
    finally:
        lib.sel_tune(26, prev)
    xr = x[:, :T].double().clone()
    wr = w.double().clone().requires_grad_(True)
    pre = torch.nn.functional.conv1d(xr.permute(0, 2, 1), wr, None, stride=s, padding=pad).permute(0, 2, 1)
    pre.backward(g[:, :T_out].double())
    rel = lambda a, r: ((a.double() - r).norm() / r.norm()).item()  # noqa: E731
    assert rel(gw, wr.grad) <= 1e-4, (tag, rel(gw, wr.grad))
    assert rel(gw1, wr.grad) <= 1e-4, (tag, rel(gw1, wr.grad))
    gbr = g[:, :T_out].double().sum((0, 1))
    assert rel(gb, gbr) <= 1e-5 and rel(gb1, gbr) <= 1e-5


GROUPED_LAYERS = [
    ("msd1_g4_s2", 128, 128, 41, 2, 20, 4, 2, 6000),
    ("msd2_g16_s2", 128, 256, 41, 2, 20, 16, 2, 3000),
    ("msd3_g16_s4", 256, 512, 41, 4, 20, 16, 2, 1500),
    ("msd4_g16_s4", 512, 1024, 41, 4, 20, 16, 4, 752),
    ("msd5_g16_s1", 1024, 1024, 41, 1, 20, 16, 4, 188),
]


@pytest.mark.parametrize("shape", GROUPED_LAYERS, ids=[s[0] for s in GROUPED_LAYERS])
def test_grouped_prefetch_bit_identical(gpu, shape):
    """k_dconv_gpf (register-prefetched stages, default) gives the same bits as
    the synchronous k_dconv_mfma (tune key 30 = 1) for the MSD's grouped,
    strided 41-tap layers, forward (bias + LeakyReLU) and adjoint (So phases)."""
    from sel import _lib as Lb
    lib = Lb.lib()
    tag, cin, cout, Kt, s, pad, G, Bs, T = shape
    from sel import dconvops as DC
    sp = DC.LayerSpec(cin, cout, Kt, s, pad, G, True)
    torch.manual_seed(Kt * 3 + cout + G)
    T_out = sp.t_out(T)
    Ta = DC._roundup(T, s)
    x = torch.zeros(Bs, Ta, cin, device=gpu)
    x[:, :T] = torch.randn(Bs, T, cin, device=gpu)
    x = x.to(torch.bfloat16)
    w = torch.randn(cout, cin // G, Kt, device=gpu) / (cin // G * Kt) ** 0.5
    b = torch.randn(cout, device=gpu)
    g = torch.randn(Bs, T_out, cout, device=gpu).to(torch.bfloat16)
    prev = lib.sel_tune(30, 1)
    try:
        ref = _run(sp, x, w, b, g, (Bs, T, Ta, T_out), torch.bfloat16)
        lib.sel_tune(30, 0)
        got = _run(sp, x, w, b, g, (Bs, T, Ta, T_out), torch.bfloat16)
    finally:
        lib.sel_tune(30, prev)
    for name, r, o in zip(("fwd", "adjoint"), ref, got):
        assert torch.equal(r, o), (tag, name, float((r.float() - o.float()).abs().max()))
