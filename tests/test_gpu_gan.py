"""GPU parity of GAN mode (BASELINE config C5): the HiFi-GAN
MSD + MPD discriminator (models/vocoder/HiFiGAN.py:308-395), the adversarial
and feature-matching losses, and the discriminator conv kernels (dconv.hip).

Goldens (tests/golden/discriminator.npz, gan_step.npz) come from the reference
itself at reduced width (make_goldens.py --only gan).  Tolerances: fp32 path
(v_mfma_f32_32x32x2_f32, exact fp32 products, different summation order than
MKL-DNN) 1e-5 norm-wise on feature maps, 1e-4 on gradients; bf16 path 3e-2
norm-wise against the fp32 golden.
"""
import numpy as np
import pytest
import torch

from conftest import golden

pytestmark = pytest.mark.gpu

D_PARAMS = dict(
    scales=3, scale_downsample_pooling="AvgPool1d",
    scale_downsample_pooling_params={"kernel_size": 4, "stride": 2, "padding": 2},
    scale_discriminator_params={"in_channels": 1, "out_channels": 1, "kernel_sizes": [15, 41, 5, 3],
                                "channels": 16, "max_downsample_channels": 32, "max_groups": 16, "bias": True,
                                "downsample_scales": [4, 4, 4, 4, 1], "nonlinear_activation": "LeakyReLU",
                                "nonlinear_activation_params": {"negative_slope": 0.1}},
    follow_official_norm=True, periods=[2, 3, 5, 7, 11],
    period_discriminator_params={"in_channels": 1, "out_channels": 1, "kernel_sizes": [5, 3], "channels": 4,
                                 "downsample_scales": [3, 3, 3, 3, 1], "max_downsample_channels": 32,
                                 "bias": True, "nonlinear_activation": "LeakyReLU",
                                 "nonlinear_activation_params": {"negative_slope": 0.1},
                                 "use_weight_norm": True, "use_spectral_norm": False})


def gan_cotangent(shape, i, j):
    return torch.randn(shape, generator=torch.Generator().manual_seed(1000 * i + j))


def rel(a, b):
    a = a.detach().double().cpu()
    b = torch.as_tensor(np.asarray(b)).double()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _disc(dev, g=None):
    from models.vocoder.HiFiGAN import Discriminator
    g = g or golden("discriminator")
    D = Discriminator(**D_PARAMS)
    sd = {k[3:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("sd.")}
    assert set(sd) == set(D.state_dict()), set(sd) ^ set(D.state_dict())
    D.load_state_dict(sd)
    return D.to(dev), g


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_discriminator_matches_reference_golden(gpu, dtype):
    from sel.convops import precision
    D, g = _disc(gpu)
    x = torch.from_numpy(g["x"]).to(gpu).requires_grad_(True)
    dt = torch.float32 if dtype == "fp32" else torch.bfloat16
    tol_f, tol_g = (1e-5, 1e-4) if dtype == "fp32" else (3e-2, 5e-2)
    with precision(dt):
        outs = D(x)
        assert len(outs) == 8
        tot = 0.0
        for i, o in enumerate(outs):
            for j, t in enumerate(o):
                ref = g[f"out.{i}.{j}"]
                assert tuple(t.shape) == ref.shape, (i, j, tuple(t.shape), ref.shape)
                assert rel(t, ref) <= tol_f, (i, j, rel(t, ref))
                tot = tot + (t.float() * gan_cotangent(t.shape, i, j).to(gpu)).sum()
        tot.backward()
    assert rel(x.grad, g["grad_x"]) <= tol_g, rel(x.grad, g["grad_x"])
    # parameters: all gradients concatenated within tol_g; each tensor within
    # tol_g (fp32) or 1.5e-1 (bf16: a 4-channel layer's weight_g gradient is a
    # sum of a few thousand bf16 products with heavy cancellation, 6e-2 measured)
    num = den = 0.0
    for name, p in D.named_parameters():
        ref = torch.from_numpy(g["g." + name]).double()
        num += ((p.grad.double().cpu() - ref) ** 2).sum().item()
        den += (ref ** 2).sum().item()
        assert rel(p.grad, ref) <= (tol_g if dtype == "fp32" else 1.5e-1), (name, rel(p.grad, ref))
    assert (num / den) ** 0.5 <= tol_g, (num / den) ** 0.5


def test_gan_losses_match_reference_golden(gpu):
    from losses import DiscriminatorAdversarialLoss, FeatureMatchLoss, GeneratorAdversarialLoss
    D, g = _disc(gpu)
    xs = torch.from_numpy(g["x"]).to(gpu)
    ys = torch.from_numpy(g["y"]).to(gpu)
    with torch.no_grad():
        oy = D(ys)
        ox = D(xs)
    chk = lambda v, k, t=1e-5: abs(v.item() - float(g[k])) <= t * abs(float(g[k])) + 1e-7  # noqa: E731
    assert chk(GeneratorAdversarialLoss(average_by_discriminators=False)(ox), "loss.gen_adv")
    assert chk(GeneratorAdversarialLoss()(ox), "loss.gen_adv_avg")
    assert chk(GeneratorAdversarialLoss(loss_type="hinge")(ox), "loss.gen_adv_hinge")
    rl, fl = DiscriminatorAdversarialLoss(average_by_discriminators=False)(ox, oy)
    assert chk(rl, "loss.dis_real") and chk(fl, "loss.dis_fake")
    rl, fl = DiscriminatorAdversarialLoss(loss_type="hinge")(ox, oy)
    assert chk(rl, "loss.dis_real_hinge") and chk(fl, "loss.dis_fake_hinge")
    fm = FeatureMatchLoss(average_by_discriminators=False, average_by_layers=False, include_final_outputs=False)
    assert chk(fm(ox, oy), "loss.feat_match")
    assert chk(FeatureMatchLoss()(ox, oy), "loss.feat_match_default")
    assert chk(FeatureMatchLoss(include_final_outputs=True)(ox, oy), "loss.feat_match_final")
    # gradient of the generator-side GAN terms w.r.t. the fake input
    x = xs.clone().requires_grad_(True)
    oh = D(x)
    (GeneratorAdversarialLoss(average_by_discriminators=False)(oh) + 2.0 * fm(oh, oy)).backward()
    assert rel(x.grad, g["grad_x.gen_terms"]) <= 1e-4, rel(x.grad, g["grad_x.gen_terms"])


# ---------------------------------------------------------------- kernel level
# full-width C5 layer shapes (48 kHz, B = 2 clips of 0.25 s): (tag, cin, cout, Kt, stride, pad, groups, Bs, T)
C5_LAYERS = [
    ("msd1_g4_s4", 128, 128, 41, 4, 20, 4, 2, 12000),
    ("msd2_g16_s4", 128, 256, 41, 4, 20, 16, 2, 3000),
    ("msd3_g16_s4", 256, 512, 41, 4, 20, 16, 2, 752),
    ("msd5_g16_s1", 1024, 1024, 41, 1, 20, 16, 2, 48),
    ("msd6_k5", 1024, 1024, 5, 1, 2, 1, 2, 48),
    ("mpd1_s3", 32, 128, 5, 3, 2, 1, 6, 2001),
    ("mpd3_s3", 512, 1024, 5, 3, 2, 1, 6, 75),
    ("mpd4_s1", 1024, 1024, 5, 1, 2, 1, 6, 25),
    ("msd0_c1", 1, 128, 15, 1, 7, 1, 2, 3000),
    ("mpd0_c1_s3", 1, 32, 5, 3, 2, 1, 6, 6001),
    ("msd7_n1", 1024, 1, 3, 1, 1, 1, 2, 48),
    ("mpd_out_n1", 1024, 1, 2, 1, 1, 1, 6, 25),
]


def _layer_ref(x, w, b, sp, slope, leaky=True):
    """fp64 torch conv of the same operands (B, T, C) -> (B, T_out, N)."""
    y = torch.nn.functional.conv1d(x.double().permute(0, 2, 1), w.double(), b.double(), stride=sp.stride,
                                   padding=sp.pad, groups=sp.groups)
    if leaky:
        y = torch.nn.functional.leaky_relu(y, slope)
    return y.permute(0, 2, 1)


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
@pytest.mark.parametrize("shape", C5_LAYERS, ids=[s[0] for s in C5_LAYERS])
def test_dconv_layer_fwd_dgrad_wgrad(gpu, shape, dtype):
    """One discriminator layer through the primitive (forward, adjoint, weight /
    bias gradient) against fp64 torch on the same operands, MFMA and VALU
    kernels both (tune key 9 = 1 forces the VALU kernel).  Bounds: fp32 1e-5
    (fwd) / 1e-4 (grads); bf16: operand rounding only, 1e-2 / 2e-2."""
    from sel import _lib as Lb
    from sel import dconvops as DC
    tag, cin, cout, Kt, s, pad, G, Bs, T = shape
    dt = torch.float32 if dtype == "fp32" else torch.bfloat16
    sp = DC.LayerSpec(cin, cout, Kt, s, pad, G, cout > 1)
    slope = 0.1
    torch.manual_seed(Kt * 7 + cin)
    T_out = sp.t_out(T)
    Ta = DC._roundup(T, s)
    x = torch.zeros(Bs, Ta, cin, device=gpu)
    x[:, :T] = torch.randn(Bs, T, cin, device=gpu)
    x = x.to(dt)
    w = torch.randn(cout, cin // G, Kt, device=gpu) / (cin // G * Kt) ** 0.5
    b = torch.randn(cout, device=gpu)
    wq = w.to(dt).float()  # the packed operand the kernel multiplies
    ref = _layer_ref(x[:, :T].float(), wq, b, sp, slope, sp.leaky)
    gy = torch.randn(Bs, T_out, cout, device=gpu)
    xr = x[:, :T].double().clone().requires_grad_(True)
    wr = wq.double().clone().requires_grad_(True)
    br = b.double().clone().requires_grad_(True)
    pre = torch.nn.functional.conv1d(xr.permute(0, 2, 1), wr, br, stride=s, padding=pad, groups=G).permute(0, 2, 1)
    pre.backward(gy.to(dt).double())
    tf, tg = (1e-5, 1e-4) if dtype == "fp32" else (1e-2, 2e-2)
    lib = Lb.lib()
    for force_valu in (0, 1):
        prev = lib.sel_tune(9, force_valu)
        try:
            d = DC._fwd_desc(sp, Bs, T, Ta, T_out, T_out, slope)
            y = torch.empty(Bs, T_out, cout, dtype=dt, device=gpu)
            DC.prim(d, x, DC.pack(sp, w, None, dt, 0), y, bias=b)
            e = ((y.double() - ref).norm() / ref.norm()).item()
            assert e <= tf, ("fwd", force_valu, e)
            # adjoint + weight gradient on gout = gy (no activation: the pre-activation gradient)
            g = gy.to(dt).contiguous()
            db = DC._dgrad_desc(sp, Bs, Ta, T_out, T_out, slope, False)
            gin = torch.empty(Bs, Ta, cin, dtype=dt, device=gpu)
            DC.prim(db, g, DC.pack(sp, w, None, dt, 1), gin)
            e = ((gin[:, :T].double() - xr.grad).norm() / xr.grad.norm()).item()
            assert e <= tg, ("dgrad", force_valu, e)
            gw, _, gb = DC.wgrad(sp, d, g, x, w, None, True, True)
            e = ((gw.double() - wr.grad).norm() / wr.grad.norm()).item()
            assert e <= tg, ("wgrad", force_valu, e)
            e = ((gb.double() - br.grad).norm() / br.grad.norm()).item()
            assert e <= tg, ("bias grad", force_valu, e)
        finally:
            lib.sel_tune(9, prev)


def test_weight_norm_pack_and_grad(gpu):
    """torch.nn.utils.weight_norm (the MPD's): w = g v / ||v|| packed on device,
    and (dL/dv, dL/dg) from the fused wgrad reduction vs torch autograd."""
    from sel import dconvops as DC
    sp = DC.LayerSpec(32, 128, 5, 3, 2, 1, True)
    torch.manual_seed(3)
    v = torch.randn(128, 32, 5, device=gpu)
    gn = torch.rand(128, device=gpu) + 0.5
    Bs, T = 3, 300
    x = torch.randn(Bs, T, 32, device=gpu)
    T_out = sp.t_out(T)
    d = DC._fwd_desc(sp, Bs, T, T, T_out, T_out, 0.1)
    y = torch.empty(Bs, T_out, 128, device=gpu)
    DC.prim(d, x, DC.pack(sp, v, gn, torch.float32, 0), y)
    vr = v.double().clone().requires_grad_(True)
    gr = gn.double().clone().requires_grad_(True)
    wr = gr.view(-1, 1, 1) * vr / vr.flatten(1).norm(dim=1).view(-1, 1, 1)
    pre = torch.nn.functional.conv1d(x.double().permute(0, 2, 1), wr, stride=3, padding=2).permute(0, 2, 1)
    ref = torch.nn.functional.leaky_relu(pre, 0.1)
    assert ((y.double() - ref).norm() / ref.norm()).item() < 1e-5
    gy = torch.randn_like(pre)
    pre.backward(gy)
    gv, gg, _ = DC.wgrad(sp, d, gy.float().contiguous(), x, v, gn, True, False)
    assert ((gv.double() - vr.grad).norm() / vr.grad.norm()).item() < 1e-4
    assert ((gg.double() - gr.grad).norm() / gr.grad.norm()).item() < 1e-4


def test_mpd_fold_and_avgpool_adjoints(gpu):
    """Front-ends: reflect-pad period fold and AvgPool1d(4, 2, 2) vs torch, and
    their adjoints via <A x, y> = <x, A^T y>."""
    from sel import dconvops as DC
    torch.manual_seed(0)
    for T, p in ((1200, 7), (1200, 11), (4801, 2), (999, 5)):
        x = torch.randn(2, T, device=gpu)
        L = (T + p - 1) // p
        y = DC.MpdFoldFn.apply(x, p, DC._roundup(L, 3))
        xp = torch.nn.functional.pad(x.view(2, 1, T), (0, L * p - T), "reflect") if T % p else x.view(2, 1, T)
        ref = xp.view(2, L, p).permute(0, 2, 1).reshape(2 * p, L)
        assert torch.equal(y[:, :L], ref) and not y[:, L:].any()
        xg = x.clone().requires_grad_(True)
        gy = torch.randn_like(y)
        (DC.MpdFoldFn.apply(xg, p, y.shape[1]) * gy).sum().backward()
        lhs = (y * gy).sum().double()
        rhs = (x * xg.grad).sum().double()
        assert abs(lhs - rhs) <= 1e-4 * abs(lhs), (T, p)
    x = torch.randn(3, 4801, device=gpu, requires_grad=True)
    y = DC.AvgPoolFn.apply(x, 4, 2, 2)
    ref = torch.nn.functional.avg_pool1d(x.view(3, 1, -1), 4, 2, 2).view(3, -1)
    assert torch.allclose(y, ref, atol=1e-6)
    gy = torch.randn_like(y)
    y.backward(gy)
    xr = x.detach().clone().requires_grad_(True)
    torch.nn.functional.avg_pool1d(xr.view(3, 1, -1), 4, 2, 2).view(3, -1).backward(gy)
    assert torch.allclose(x.grad, xr.grad, atol=1e-6)


def _adam_update_check(before, after_ref_prev, after_ref, p_now, lr):
    """Adam's first steps move each weight by about +-lr * sign(g): a weight whose
    tiny gradient flips sign under fp32 reordering moves 2 lr the other way.
    Returns (#flipped, #total, squared error, squared norm) of the update."""
    ref = after_ref.double() - after_ref_prev.double()
    d = (p_now.detach().double().cpu() - before.double())
    return (((d - ref).abs() > 0.5 * lr).sum().item(), d.numel(), ((d - ref) ** 2).sum().item(),
            (ref ** 2).sum().item())


def test_gan_step_matches_reference_golden(gpu):
    """Two GAN-mode train_denoise steps (:138-165, :213-263, discriminator
    enabled) on the reduced-width without-PQC generator + discriminator, fp32,
    against the reference's own run (tests/golden/gan_step.npz): the loss terms
    to 1e-5 (step 0) / 1e-4 (step 1), and each network's Adam update with at most
    2% sign-flipped weights and <= 10% norm-wise update error (as
    test_gpu_glue.test_train_step_matches_golden explains)."""
    from models.autoencoder_without_PQC.AudioDec import Generator
    from sel import configs
    from train_denoise import DenoiseStep
    g = golden("gan_step")
    gp = dict(encode_channels=4, decode_channels=4, code_dim=64, codebook_num=2, codebook_size=64)
    G = Generator(**gp)
    G.load_state_dict({k[3:]: torch.from_numpy(v) for k, v in golden("generator_nopqc").items()
                       if k.startswith("sd.")})
    D, _ = _disc(gpu)
    G = G.to(gpu)
    cfg = configs.get("symAD_vctk_48000_hop300")
    step = DenoiseStep(cfg, gpu, generator=G, discriminator=D)
    step.discriminator_enabled = True
    x, y = torch.from_numpy(g["x_noisy"]), torch.from_numpy(g["x_clean"])
    prev_g = {k: p.detach().cpu().clone() for k, p in G.named_parameters()}
    prev_d = {k: p.detach().cpu().clone() for k, p in D.named_parameters()}
    for s in range(2):
        bg = {k: p.detach().cpu().clone() for k, p in G.named_parameters()}
        bd = {k: p.detach().cpu().clone() for k, p in D.named_parameters()}
        gen, dis, frags = step.model_step(y, x)
        tol = 1e-5 if s == 0 else 1e-4
        f = dict(frags)
        for name, v in (("gen", gen), ("dis", dis), ("mel", f["mel_loss"]), ("adv", f["adv_loss"]),
                        ("fm", f["feat_loss"])):
            ref = float(g[f"{name}.{s}"])
            assert abs(v.item() - ref) <= tol * abs(ref) + 1e-7, (s, name, v.item(), ref)
        for net, before, prev, key, lr in ((G, bg, prev_g, "g_sd", 1e-4), (D, bd, prev_d, "d_sd", 2e-4)):
            flips = tot = num = den = 0
            for k, p in net.named_parameters():
                if f"{key}{s + 1}.{k}" not in g:
                    continue
                ref_now = torch.from_numpy(g[f"{key}{s + 1}.{k}"])
                a, b_, c, d_ = _adam_update_check(before[k], prev[k] if s == 0 else
                                                  torch.from_numpy(g[f"{key}{s}.{k}"]), ref_now, p, lr)
                flips, tot, num, den = flips + a, tot + b_, num + c, den + d_
                with torch.no_grad():  # continue from the reference's weights
                    p.copy_(ref_now.to(gpu))
            assert tot > 0 and flips <= 0.02 * tot, (s, key, flips, tot)
            assert (num / den) ** 0.5 <= 0.10, (s, key, (num / den) ** 0.5)


def test_gan_step_bf16_runs_and_tracks_fp32(gpu):
    """The same GAN step in bf16 (C5's precision): finite, and its loss terms
    within 3e-2 of the fp32 step's on the same weights."""
    from models.autoencoder_without_PQC.AudioDec import Generator
    from sel import configs
    from sel.convops import precision
    from train_denoise import DenoiseStep
    g = golden("gan_step")
    gp = dict(encode_channels=4, decode_channels=4, code_dim=64, codebook_num=2, codebook_size=64)
    x, y = torch.from_numpy(g["x_noisy"]), torch.from_numpy(g["x_clean"])
    vals = []
    for dt in (torch.float32, torch.bfloat16):
        G = Generator(**gp)
        G.load_state_dict({k[3:]: torch.from_numpy(v) for k, v in golden("generator_nopqc").items()
                           if k.startswith("sd.")})
        D, _ = _disc(gpu)
        step = DenoiseStep(configs.get("symAD_vctk_48000_hop300"), gpu, generator=G.to(gpu), discriminator=D)
        step.discriminator_enabled = True
        with precision(dt):
            gen, dis, frags = step.model_step(y, x)
        vals.append([gen.item(), dis.item()] + [float(v) for _, v in frags[:3]])
    for a, b in zip(vals[1], vals[0]):
        assert np.isfinite(a) and abs(a - b) <= 3e-2 * abs(b) + 1e-6, (vals[1], vals[0])


@pytest.mark.parametrize("dt", ["fp32", "bf16"])
def test_gan_step_reused_real_half_matches_concatenated(gpu, dt, monkeypatch):
    """The D step's real half reused from the generator step
    (DenoiseStep._reuse_real: Discriminator.stash_first_half, then
    forward_second_half) against ONE pass over the concatenated batch
    (SEL_REUSE_REAL=0): same losses and the same discriminator gradients.  Both
    run the same kernels per clip; the flat tiling may place the clips in
    other tiles, so the bar is 1e-6 (fp32) / 1e-3 (bf16) norm-wise, not bit
    equality."""
    from models.autoencoder_without_PQC.AudioDec import Generator
    from sel import configs
    from sel.convops import precision
    from train_denoise import DenoiseStep
    g = golden("gan_step")
    gp = dict(encode_channels=4, decode_channels=4, code_dim=64, codebook_num=2, codebook_size=64)
    x, y = torch.from_numpy(g["x_noisy"]), torch.from_numpy(g["x_clean"])
    res = []
    for reuse in ("0", "1"):
        monkeypatch.setenv("SEL_REUSE_REAL", reuse)
        G = Generator(**gp)
        G.load_state_dict({k[3:]: torch.from_numpy(v) for k, v in golden("generator_nopqc").items()
                           if k.startswith("sd.")})
        G = G.to(gpu)
        D, _ = _disc(gpu)
        step = DenoiseStep(configs.get("symAD_vctk_48000_hop300"), gpu, generator=G, discriminator=D)
        step.discriminator_enabled = True
        assert step._reuse_real() == (reuse == "1")
        # no optimizer update: compare the gradients the D step leaves
        step.optimizer["discriminator"].step = lambda *a, **k: None
        with precision(torch.float32 if dt == "fp32" else torch.bfloat16):
            gen, dis, frags = step.model_step(y, x)
        torch.cuda.synchronize()
        res.append(([gen.item(), dis.item()] + [float(v) for _, v in frags[:3]],
                    [p.grad.detach().double().clone() for p in D.parameters()]))
    tol = 1e-6 if dt == "fp32" else 1e-3
    for a, b in zip(res[1][0], res[0][0]):
        assert abs(a - b) <= tol * abs(b) + 1e-9, (res[1][0], res[0][0])
    num = sum(((a - b) ** 2).sum().item() for a, b in zip(res[1][1], res[0][1]))
    den = sum((b ** 2).sum().item() for b in res[0][1])
    exact = all(torch.equal(a, b) for a, b in zip(res[1][1], res[0][1]))
    print(f"reuse vs concatenated ({dt}): grad rel {(num / den) ** 0.5:.3e}, bit-equal {exact}")
    assert (num / den) ** 0.5 <= tol, (num / den) ** 0.5


@pytest.mark.parametrize("dt", ["fp32", "bf16"])
def test_gan_step_side_streams_bit_identical_to_serial(gpu, dt, monkeypatch):
    """The sub-discriminator chains on side streams (sel.streams, SEL_D_STREAMS)
    against everything on one stream: the same kernels in the same order per
    chain, so the losses and the generator and discriminator gradients are
    bit-identical (twice with streams on: a missing stream dependency would
    show up as a difference from the serial run), and with the chains' final
    weight-gradient reductions as one launch per layer instead of one per chain
    (sel_dconv_wgrad vs sel_dconv_wgrad_finish_many: the same per-channel
    reduction)."""
    from models.autoencoder_without_PQC.AudioDec import Generator
    from sel import configs
    from sel import dconvops
    from sel.convops import precision
    from train_denoise import DenoiseStep
    g = golden("gan_step")
    gp = dict(encode_channels=4, decode_channels=4, code_dim=64, codebook_num=2, codebook_size=64)
    x, y = torch.from_numpy(g["x_noisy"]), torch.from_numpy(g["x_clean"])
    res = []
    for n_streams, merge in (("0", True), ("8", True), ("2", True), ("8", True), ("0", False), ("8", False)):
        monkeypatch.setenv("SEL_D_STREAMS", n_streams)
        monkeypatch.setattr(dconvops, "DWGRAD_MERGE", merge)
        G = Generator(**gp)
        G.load_state_dict({k[3:]: torch.from_numpy(v) for k, v in golden("generator_nopqc").items()
                           if k.startswith("sd.")})
        G = G.to(gpu)
        D, _ = _disc(gpu)
        step = DenoiseStep(configs.get("symAD_vctk_48000_hop300"), gpu, generator=G, discriminator=D)
        step.discriminator_enabled = True
        step.optimizer["discriminator"].step = lambda *a, **k: None
        step.optimizer["generator"].step = lambda *a, **k: None
        with precision(torch.float32 if dt == "fp32" else torch.bfloat16):
            gen, dis, frags = step.model_step(y, x)
        torch.cuda.synchronize()
        res.append(([gen.item(), dis.item()] + [float(v) for _, v in frags[:3]],
                    [p.grad.detach().clone() for p in list(D.parameters()) + list(G.parameters())
                     if p.grad is not None]))
    for r in res[1:]:
        assert r[0] == res[0][0], (r[0], res[0][0])
        assert len(r[1]) == len(res[0][1]) > 0
        assert all(torch.equal(a, b) for a, b in zip(r[1], res[0][1]))
