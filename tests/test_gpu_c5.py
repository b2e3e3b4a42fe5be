"""Parity of the C5 (BASELINE configs[4]) GAN-mode path at the bench's own size:
B = 16 clips x 1 s @ 48 kHz, symAD_vctk_48000_hop300, full-width HiFi-GAN MSD +
MPD (models/vocoder/HiFiGAN.py:308-395, modules/discriminator.py:26-447).

1. Every MPD layer that takes the warp-specialised kernel (conv.hip
   k_conv_ws_bf16 via dconv_ws_fwd) at C5 sizes, forward and adjoint, in the
   period chain's own zero-gapped layout (sel.dconvops.period_alloc /
   chain_layout, one row pitch per layer): the launcher must report the FLAT
   tiling (include/sel.h SEL_DPATH_WS_FLAT) — so the test cannot pass on a
   fallback — and the result must match fp64 torch on the same bf16 operands
   and be bit-identical to the per-sequence tiles (tune key 22 = 1, same MFMA
   order per output) and, on the 512 / 1024-wide layers, to the 12-wave kernel
   (tune key 37 = 1; the default there is the eight-wave k_conv_ws8).  The adjoint's gradient gap rows hold NaN: they must
   never be read.  Both G-step (16 clips) and D-step (32 clips) batches.
2. A full-chain backward whose feature-map gradients live in NaN-filled
   buffers (what GanReduceFn.backward hands over: only the view is written)
   gives the same bits as with zero-filled buffers.
3. One full-width GAN step, bf16 and fp32, against the fp32 oracle
   (oracle/ref_ops.py, run by torch on the same GPU with MIOpen off: native
   im2col + BLAS, no kernel of ours) on the same weights and inputs
   (train_denoise.py:138-165, :213-263): generator output, every D feature
   map, the mel / adv / feature-matching terms, the D loss, and gradients by
   the same-upstream technique of test_gpu_c3.py (each side back-propagates
   the ORACLE's upstream gradient, isolating each backward).
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

CFG = "symAD_vctk_48000_hop300"
CLIPS = 16
T48 = 48000
PERIODS = (2, 3, 5, 7, 11)
SLOPE = 0.1


def _mpd_specs():
    from oracle import ref_ops as R
    from sel import configs
    from sel import dconvops as DC
    pp = configs.get(CFG)["discriminator_params"]["period_discriminator_params"]
    return [DC.LayerSpec(ci, co, k, s, p, 1, lk) for (ci, co, k, s, p, lk) in R.period_discriminator_plan(**pp)]


def _check(got, ref, what):
    """bf16 output rounding bound (test_gpu_c3.py): <= 4e-3 norm-wise and
    elementwise |a-b| <= 8e-3|b| + 2e-3 max|b|."""
    g = got.double()
    e = ((g - ref).norm() / ref.norm()).item()
    assert e <= 4e-3, (what, e)
    bad = (g - ref).abs() > 8e-3 * ref.abs() + 2e-3 * ref.abs().max()
    assert not bad.any(), (what, int(bad.sum()), (g - ref).abs().max().item())


@pytest.mark.parametrize("clips", [CLIPS, 2 * CLIPS], ids=["g_step", "d_step"])
@pytest.mark.parametrize("period", PERIODS)
def test_mpd_ws_flat_layers_at_c5_shapes(gpu, period, clips):
    from sel import _lib as Lb
    from sel import dconvops as DC
    lib = Lb.lib()
    dt = torch.bfloat16
    specs = _mpd_specs()
    Lv = (T48 + period - 1) // period
    Bs = clips * period
    geo = DC.chain_layout(specs, Lv, DC.period_alloc(Lv, specs))
    gen = torch.Generator(device=gpu).manual_seed(1000 * period + clips)
    n_flat = 0
    for li, (sp, (T_in, Ta, T_out, To)) in enumerate(zip(specs, geo)):
        d = DC._fwd_desc(sp, Bs, T_in, Ta, T_out, To, SLOPE)
        db = DC._dgrad_desc(sp, Bs, Ta, T_out, To, SLOPE, li > 0, T_in=T_in)
        fwd_ws, adj_ws = DC.kernel(d, dt)[0] == "ws_flat", DC.kernel(db, dt)[0] == "ws_flat"
        if not (fwd_ws or adj_ws):
            continue
        s = sp.stride
        x = torch.zeros(Bs, Ta, sp.cin, device=gpu)
        x[:, :T_in] = torch.randn(Bs, T_in, sp.cin, generator=gen, device=gpu)
        x = x.to(dt)
        w = torch.randn(sp.cout, sp.cin, sp.Kt, generator=gen, device=gpu) / (sp.cin * sp.Kt) ** 0.5
        b = torch.randn(sp.cout, generator=gen, device=gpu)
        wq = w.to(dt).double()
        if fwd_ws:
            n_flat += 1
            pre = torch.nn.functional.conv1d(x[:, :T_in].double().permute(0, 2, 1), wq, b.double(), stride=s,
                                             padding=sp.pad).permute(0, 2, 1)
            ref = torch.nn.functional.leaky_relu(pre, SLOPE)
            ys = []
            for flat_off, ws8_off in ((0, 0), (1, 0), (0, 1)):
                prev, prev8 = lib.sel_tune(22, flat_off), lib.sel_tune(37, ws8_off)
                try:
                    assert DC.kernel(d, dt)[0] == ("ws" if flat_off else "ws_flat"), (li, flat_off)
                    y = torch.full((Bs, To, sp.cout), 7.0, dtype=dt, device=gpu)
                    DC.prim(d, x, DC._pack(sp, w, None, dt, 0), y, bias=b)
                finally:
                    lib.sel_tune(22, prev)
                    lib.sel_tune(37, prev8)
                ys.append(y)
            _check(ys[0][:, :T_out], ref, (period, clips, li, "fwd"))
            assert torch.count_nonzero(ys[0][:, T_out:]).item() == 0, (li, "rows past T_out")
            assert torch.equal(ys[0], ys[1]), (li, "flat vs per-sequence tiles")
            assert torch.equal(ys[0], ys[2]), (li, "eight-wave vs 12-wave kernel")
        if adj_ws:
            n_flat += 1
            g = torch.full((Bs, To, sp.cout), float("nan"), device=gpu)
            g[:, :T_out] = torch.randn(Bs, T_out, sp.cout, generator=gen, device=gpu)
            g = g.to(dt)
            aux = torch.randn(Bs, Ta, sp.cin, generator=gen, device=gpu).to(dt)
            res = torch.randn(Bs, Ta, sp.cin, generator=gen, device=gpu).to(dt)
            xr = torch.zeros(Bs, T_in, sp.cin, dtype=torch.float64, device=gpu, requires_grad=True)
            torch.nn.functional.conv1d(xr.permute(0, 2, 1), wq, None, stride=s, padding=sp.pad).permute(
                0, 2, 1).backward(g[:, :T_out].double())
            ref = (xr.grad + res[:, :T_in].double()) * torch.where(aux[:, :T_in].double() > 0, 1.0, SLOPE)
            gs = []
            for flat_off, ws8_off in ((0, 0), (1, 0), (0, 1)):
                prev, prev8 = lib.sel_tune(22, flat_off), lib.sel_tune(37, ws8_off)
                try:
                    assert DC.kernel(db, dt)[0] == ("ws" if flat_off else "ws_flat"), (li, flat_off)
                    gin = torch.full((Bs, Ta, sp.cin), 7.0, dtype=dt, device=gpu)
                    DC.prim(db, g, DC._pack(sp, w, None, dt, 1), gin, aux=aux, res=res)
                finally:
                    lib.sel_tune(22, prev)
                    lib.sel_tune(37, prev8)
                gs.append(gin)
            _check(gs[0][:, :T_in], ref, (period, clips, li, "adjoint"))
            tail = (T_in + s - 1) // s * s
            assert torch.count_nonzero(gs[0][:, tail:]).item() == 0, (li, "phase rows past the input")
            assert torch.equal(gs[0], gs[1]), (li, "adjoint flat vs per-sequence tiles")
            assert torch.equal(gs[0], gs[2]), (li, "adjoint eight-wave vs 12-wave kernel")
    torch.cuda.synchronize()
    # at C5 sizes layers 1-4 forward and 2-4 adjoint are on the flat tiles (SEL_DPATH_WS_FLAT)
    assert n_flat >= 7, n_flat


def _nan_buffer_grads(outs, cots, fill):
    """Cotangents placed like GanReduceFn.backward does: a buffer the size of the
    view's base, only the view written, the rest `fill`."""
    grads = []
    for o, c in zip(outs, cots):
        base = o._base if o._base is not None else o
        if base is o:
            grads.append(c)
            continue
        buf = torch.full_like(base, fill)
        ga = torch.as_strided(buf, o.shape, o.stride(), o.storage_offset())
        ga.copy_(c)
        grads.append(ga)
    return grads


@pytest.mark.parametrize("which", ["mpd_p2", "mpd_p11", "msd0"])
def test_gap_rows_of_feature_map_grads_are_never_read(gpu, which):
    from models.vocoder.HiFiGAN import Discriminator
    from sel import configs
    from sel.convops import precision
    import warnings
    dp = configs.get(CFG)["discriminator_params"]
    torch.manual_seed(5)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        Dm = Discriminator(**dp).to(gpu)
    sub = Dm.mpd.discriminators[PERIODS.index(int(which[5:]))] if which.startswith("mpd") \
        else Dm.msd.discriminators[0]
    x = 0.1 * torch.randn(4, 1, T48, device=gpu)
    res = []
    with precision(torch.bfloat16):
        for fill in (0.0, float("nan")):
            xi = x.clone().requires_grad_(True)
            for p in sub.parameters():
                p.grad = None
            outs = sub(xi)
            g = torch.Generator(device=gpu).manual_seed(9)
            cots = [torch.randn(o.shape, generator=g, device=gpu).to(o.dtype) for o in outs]
            torch.autograd.backward(outs, _nan_buffer_grads(outs, cots, fill))
            res.append([xi.grad.clone()] + [p.grad.clone() for p in sub.parameters()])
    for a, b in zip(*res):
        assert torch.isfinite(b).all()
        assert torch.equal(a, b), which


def _oracle_step(cfg, PG, PD, x, clean, pred_fixed):
    """fp32 oracle of the generator loss (with its gradients w.r.t. the trainable
    generator weights and w.r.t. the waveform) and of the D loss on a fixed
    prediction (with the D weight gradients)."""
    from oracle import ref_ops as R
    from oracle.melfilters import mel as melbank
    mp = cfg["mel_loss_params"]
    dkw = cfg["discriminator_params"]
    dev = x.device
    mm = torch.from_numpy(melbank(sr=mp["fs"], n_fft=2048, n_mels=80, fmin=mp["fmin"], fmax=mp["fmax"]).T.copy())
    mm, win = mm.to(dev), R.hann(2048).to(dev)
    geo = R.generator_geometry(**cfg["generator_params"])
    out = {}
    with torch.backends.cudnn.flags(enabled=False):
        pred = R.generator_forward(PG, x, geo, pqc=False)
        pred.retain_grad()
        mel = R.multi_mel_loss(pred, clean, [(2048, 300, 2048)], [win], [mm], 1e-10, None)
        d_hat = R.hifigan_discriminator(PD, pred, **dkw)
        with torch.no_grad():
            d_real = R.hifigan_discriminator(PD, clean, **dkw)
        adv = R.generator_adv_loss(pred, False)  # train_denoise.py:147 passes the waveform
        fm = R.feat_match_loss(d_hat, d_real)
        gen = cfg["lambda_mel_loss"] * mel + cfg["lambda_adv"] * adv + cfg["lambda_feat_match"] * fm
        gen.backward()
        out.update(pred=pred.detach(), mel=mel.item(), adv=adv.item(), fm=fm.item(), gen=gen.item(),
                   gy=pred.grad.detach().clone(), d_hat=[[t.detach() for t in o] for o in d_hat])
        out["g_grads"] = {k: v.grad.detach().clone() for k, v in PG.items() if v.grad is not None}
        for v in PD.values():
            v.requires_grad_(True)
        rl, fl = R.discriminator_adv_loss(R.hifigan_discriminator(PD, pred_fixed, **dkw),
                                          R.hifigan_discriminator(PD, clean, **dkw), False)
        dis = cfg["lambda_adv"] * (rl + fl)
        dis.backward()
        out["dis"] = dis.item()
        out["d_grads"] = {k: v.grad.detach().clone() for k, v in PD.items()}
    return out


def _rel(a, b):
    return ((a.detach().double() - b.detach().double()).norm() / b.detach().double().norm().clamp_min(1e-30)).item()


def _grad_err(named, ref):
    num = den = 0.0
    worst = (0.0, "")
    for k, r in ref.items():
        gd = named[k].grad
        assert gd is not None, k
        num += ((gd.double() - r.double()) ** 2).sum().item()
        den += (r.double() ** 2).sum().item()
        worst = max(worst, (_rel(gd, r), k))
    return (num / den) ** 0.5, worst


@pytest.mark.parametrize("dtype", ["bf16", "fp32"])
def test_c5_gan_step_vs_fp32_oracle(gpu, dtype):
    """Full-width C5 GAN step pieces vs the fp32 oracle.  Bounds — fp32 (exact
    fp32 products, other summation order): 1e-4 forward / losses, 2e-3
    gradients.  bf16 (2^-9 operand rounding per layer, ~30 generator + 7-8
    discriminator layers): generator output 3e-2, D feature maps 5e-2 each,
    losses 2e-2 (mel 5e-3), gradients 5e-2 concatenated / 1e-1 worst tensor."""
    import warnings
    from dataloader.data_utils import add_noise
    from models.autoencoder_without_PQC.AudioDec import Generator
    from models.vocoder.HiFiGAN import Discriminator
    from sel import configs
    from sel.convops import precision
    from train_denoise import DenoiseStep
    cfg = configs.get(CFG)
    torch.manual_seed(93)
    G = Generator(**cfg["generator_params"])
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        D = Discriminator(**cfg["discriminator_params"])
    for mod in (G.projector, G.quantizer, G.decoder.conv1):  # unused by the without-PQC forward
        for p in mod.parameters():
            p.requires_grad_(False)
    gtrain = [k for k, p in G.named_parameters() if p.requires_grad]
    PG = {k: v.detach().clone().to(gpu) for k, v in G.state_dict().items()}
    for k in gtrain:
        PG[k].requires_grad_(True)
    PD = {k: v.detach().clone().to(gpu) for k, v in D.state_dict().items()}
    g = torch.Generator().manual_seed(17)
    clean = (0.1 * torch.randn(CLIPS, 1, T48, generator=g)).to(gpu)
    noise = (0.1 * torch.randn(CLIPS, 1, T48, generator=g)).to(gpu)
    x = add_noise(clean, noise, 15)
    # the D step's fake batch: a fixed waveform (the generator after its Adam step
    # in the real step), the same on both sides
    pred_fixed = (0.05 * torch.randn(CLIPS, 1, T48, generator=g)).to(gpu)
    ref = _oracle_step(cfg, PG, PD, x, clean, pred_fixed)

    G, D = G.to(gpu), D.to(gpu)
    step = DenoiseStep(cfg, gpu, generator=G, discriminator=D)
    step.discriminator_enabled = True
    gparams, dparams = dict(G.named_parameters()), dict(D.named_parameters())
    fp32 = dtype == "fp32"
    t_fwd, t_map, t_loss, t_mel = (1e-4, 1e-4, 1e-4, 1e-4) if fp32 else (3e-2, 5e-2, 2e-2, 5e-3)
    t_g, t_gw = (2e-3, 5e-3) if fp32 else (5e-2, 1e-1)
    with precision(torch.float32 if fp32 else torch.bfloat16):
        # generator forward, and its backward from the oracle's dL/dpred
        pred = G(x)
        e_pred = _rel(pred, ref["pred"])
        (pred * ref["gy"]).sum().backward()
        eg, worst_g = _grad_err(gparams, ref["g_grads"])
        # D forward on the oracle's prediction: every feature map
        xp = ref["pred"].clone().requires_grad_(True)
        worst_map = (0.0, "")
        with torch.no_grad():
            outs = D(ref["pred"])
        for i, (oo, rr) in enumerate(zip(outs, ref["d_hat"])):
            for j, (a, r) in enumerate(zip(oo, rr)):
                worst_map = max(worst_map, (_rel(a.reshape(r.shape), r), f"D{i}.{j}"))
        # generator loss terms on the oracle's prediction and their gradient w.r.t. it
        gen, frags = step.calculate_generator_loss(xp, clean)
        gen.backward()
        f = dict(frags)
        e_mel = abs(float(f["mel_loss"]) / cfg["lambda_mel_loss"] - ref["mel"]) / abs(ref["mel"])
        e_adv = abs(float(f["adv_loss"]) / cfg["lambda_adv"] - ref["adv"]) / abs(ref["adv"])
        e_fm = abs(float(f["feat_loss"]) / cfg["lambda_feat_match"] - ref["fm"]) / abs(ref["fm"])
        e_gy = _rel(xp.grad, ref["gy"])
        # D step on the fixed prediction
        for p in D.parameters():
            p.grad = None
        dis = step.calculate_discriminator_loss(pred_fixed, clean)
        dis.backward()
        e_dis = abs(dis.item() - ref["dis"]) / abs(ref["dis"])
        ed, worst_d = _grad_err(dparams, ref["d_grads"])
    torch.cuda.synchronize()
    print(f"C5 {dtype} vs fp32 oracle: pred {e_pred:.2e} | maps worst {worst_map} | mel {e_mel:.2e} adv {e_adv:.2e} "
          f"fm {e_fm:.2e} dis {e_dis:.2e} | dL/dpred {e_gy:.2e} | G grads {eg:.2e} worst {worst_g} | "
          f"D grads {ed:.2e} worst {worst_d}")
    assert math.isfinite(gen.item()) and math.isfinite(dis.item())
    assert e_pred <= t_fwd, e_pred
    assert worst_map[0] <= t_map, worst_map
    assert e_mel <= t_mel and e_adv <= t_loss and e_fm <= t_loss and e_dis <= t_loss, (e_mel, e_adv, e_fm, e_dis)
    assert e_gy <= t_g, e_gy
    assert eg <= t_g and worst_g[0] <= t_gw, (eg, worst_g)
    assert ed <= t_g and worst_d[0] <= t_gw, (ed, worst_d)
