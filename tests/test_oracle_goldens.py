"""Pin the CPU oracle (oracle/) against golden vectors made from the reference.

The fixtures under tests/golden/ were produced by tests/golden/make_goldens.py,
which imports the reference from /root/reference.  The oracle is a functional
PyTorch-CPU restatement; here it must reproduce those vectors (same library,
same op order -> tight tolerances)."""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle import melfilters, ref_ops as R


def _arr(a):
    return a.detach().cpu().numpy() if isinstance(a, torch.Tensor) else np.asarray(a)


def close(a, b, rtol=1e-5, atol=1e-6):
    np.testing.assert_allclose(_arr(a), _arr(b), rtol=rtol, atol=atol)


def T(a):
    return torch.from_numpy(np.asarray(a))


def test_melfilters_match_reference_buffers():
    g = golden("melmat")
    cfgs = {"24k_fmax24000": (24000, 2048, 80, 0, 24000), "24k_fmax12000": (24000, 2048, 80, 0, 12000),
            "48k_fmax24000": (48000, 2048, 80, 0, 24000), "default": (22050, 1024, 80, 80, 7600)}
    for k, (sr, n, m, lo, hi) in cfgs.items():
        mm = melfilters.mel(sr=sr, n_fft=n, n_mels=m, fmin=lo, fmax=hi).T
        np.testing.assert_array_equal(mm, g[f"melmat.{k}"])
    # the 24 kHz fmax=24000 config has 12 all-zero filters (SURVEY §7 hard part 7)
    empty = np.where(g["melmat.24k_fmax24000"].sum(0) == 0)[0]
    assert list(empty) == list(range(68, 80))


def test_stft_mag_and_losses():
    g = golden("stft")
    x, y = T(g["x"]), T(g["y"])
    for n, h, w in [(1024, 120, 600), (2048, 240, 1200), (512, 50, 240)]:
        win = R.hann(w)
        close(R.stft_mag(x, n, h, w, win), g[f"mag.{n}"])
        sc, mg = R.stft_loss(x, y, n, h, w, win)
        close(sc, g[f"sc.{n}"])
        close(mg, g[f"logmag.{n}"])
    res = [(1024, 120, 600), (2048, 240, 1200), (512, 50, 240)]
    xg = x.clone().requires_grad_(True)
    sc, mg = R.mr_stft_loss(xg.unsqueeze(1), y.unsqueeze(1), res, [R.hann(w) for _, _, w in res])
    (sc + mg).backward()
    close(sc, g["mr.sc"])
    close(mg, g["mr.mag"])
    close(xg.grad, g["mr.grad_x"], rtol=1e-4, atol=1e-7)
    close(R.stft_mag(T(g["short.x"]), 2048, 240, 1200, R.hann(1200)), g["short.mag.2048"])


def test_mel_loss():
    g = golden("mel")
    gm = golden("melmat")
    yh, y = T(g["y_hat"]), T(g["y"])
    mm = T(gm["melmat.24k_fmax24000"])
    res = [(2048, 300, 2048)]
    close(R.melspec(yh, 2048, 300, 2048, R.hann(2048), mm, 1e-10, None), g["mel24.y_hat"], rtol=1e-5, atol=1e-5)
    yg = yh.clone().requires_grad_(True)
    loss = R.multi_mel_loss(yg, y, res, [R.hann(2048)], [mm], 1e-10, None)
    loss.backward()
    close(loss, g["mel24.loss"])
    close(yg.grad, g["mel24.grad"], rtol=1e-4, atol=1e-9)
    # default multi-resolution log10 variant
    resd = [(1024, 120, 600), (2048, 240, 1200), (512, 50, 240)]
    mms = [T(melfilters.mel(sr=22050, n_fft=n, n_mels=80, fmin=80, fmax=7600).T) for n, _, _ in resd]
    yg = yh.clone().requires_grad_(True)
    loss = R.multi_mel_loss(yg, y, resd, [R.hann(w) for _, _, w in resd], mms, 1e-10, 10.0)
    loss.backward()
    close(loss, g["meldef.loss"])
    close(yg.grad, g["meldef.grad"], rtol=1e-4, atol=1e-9)


def test_conv_layers():
    g = golden("conv")
    names = sorted({k.split(".")[0] for k in g if k.endswith(".cfg")})
    for name in names:
        cfg = g[f"{name}.cfg"]
        x = T(g[f"{name}.x"]).requires_grad_(True)
        w = T(g[f"{name}.w"]).requires_grad_(True)
        b = T(g[f"{name}.b"]).requires_grad_(True) if f"{name}.b" in g else None
        if len(cfg) == 7:
            ci, co, k, s, d, hb, t = cfg
            yv = R.causal_conv1d(x, w, b, int(s), int(d))
        else:
            ci, co, k, s, hb, t = cfg
            yv = R.causal_conv_transpose1d(x, w, b, int(s))
        close(yv, g[f"{name}.y"], rtol=1e-5, atol=1e-5)
        yv.backward(T(g[f"{name}.gy"]))
        close(x.grad, g[f"{name}.gx"], rtol=1e-5, atol=1e-5)
        close(w.grad, g[f"{name}.gw"], rtol=1e-5, atol=1e-4)
        if b is not None:
            close(b.grad, g[f"{name}.gb"], rtol=1e-5, atol=1e-4)
    x = T(g["ru.x"]).requires_grad_(True)
    w1 = T(g["ru.w1"]).requires_grad_(True)
    w2 = T(g["ru.w2"]).requires_grad_(True)
    yv = R.residual_unit(x, w1, w2, 3)
    close(yv, g["ru.y"], rtol=1e-5, atol=1e-5)
    yv.backward(T(g["ru.gy"]))
    close(x.grad, g["ru.gx"], rtol=1e-5, atol=1e-5)
    close(w1.grad, g["ru.gw1"], rtol=1e-5, atol=1e-4)
    close(w2.grad, g["ru.gw2"], rtol=1e-5, atol=1e-4)


def test_residual_vq_eval():
    g = golden("vq")
    embeds = [T(g[f"embed.{i}"]) for i in range(4)]
    z = T(g["z"]).requires_grad_(True)
    q, losses, ppls, inds = R.rvq_forward(z, embeds)
    np.testing.assert_array_equal(inds.permute(0, 1, 2).numpy(), g["fi.idx"])
    close(q, g["q"])
    close(losses, g["losses"])
    close(ppls, g["ppls"])
    ((q * T(g["r"])).sum() + losses.sum()).backward()
    close(z.grad, g["grad_z"], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("tag", ["pqc", "nopqc"])
def test_generator(tag):
    g = golden(f"generator_{tag}")
    gm = golden("melmat")
    P = {k[3:]: T(v) for k, v in g.items() if k.startswith("sd.")}
    for k, v in P.items():
        if v.dtype == torch.float32 and not k.endswith(("pad_buffer", "embed", "cluster_size", "embed_avg")):
            v.requires_grad_(True)
    geo = R.generator_geometry(encode_channels=4, decode_channels=4)
    xn, xc = T(g["x_noisy"]), T(g["x_clean"])
    mm = T(gm["melmat.24k_fmax24000"])
    mel = lambda a, b: R.multi_mel_loss(a, b, [(2048, 300, 2048)], [R.hann(2048)], [mm], 1e-10, None)
    if tag == "pqc":
        y, zq, z, vql, ppl = R.generator_forward(P, xn, geo, pqc=True, codebook_num=2)
        close(z, g["z"], rtol=1e-5, atol=1e-6)
        close(zq, g["zq"], rtol=1e-5, atol=1e-6)
        close(vql, g["vqloss"], rtol=1e-5, atol=1e-7)
        close(ppl, g["ppl"])
        loss = 45.0 * mel(y, xc) + vql.sum()
    else:
        y = R.generator_forward(P, xn, geo, pqc=False)
        loss = 45.0 * mel(y, xc)
    close(y, g["y"], rtol=1e-5, atol=1e-6)
    close(loss, g["loss"], rtol=1e-5)
    loss.backward()
    for k, v in g.items():
        if k.startswith("g."):
            close(P[k[2:]].grad, v, rtol=1e-4, atol=1e-6)


def test_add_noise():
    g = golden("add_noise")
    for snr in (10, 15, 19):
        close(R.add_noise(T(g["clean"]), T(g["noise"]), snr), g[f"mixed.{snr}"], rtol=1e-6, atol=1e-7)


def test_train_step():
    """train_denoise.py:213-243 for the without-PQC generator: 45*mel, backward,
    clip_grad_norm_(1), Adam(lr 5e-5, wd 1e-6) — two steps vs the reference's run."""
    g = golden("train_step")
    gm = golden("melmat")
    P = {k[4:]: T(v).clone() for k, v in g.items() if k.startswith("sd0.")}
    train = [k for k in P if k.startswith(("encoder.", "decoder.conv_blocks", "decoder.conv2"))
             and not k.endswith("pad_buffer")]
    for k in train:
        P[k].requires_grad_(True)
    opt = torch.optim.Adam([P[k] for k in train], lr=5e-5, weight_decay=1e-6)
    geo = R.generator_geometry(encode_channels=4, decode_channels=4)
    mm = T(gm["melmat.24k_fmax24000"])
    xn, xc = T(g["x_noisy"]), T(g["x_clean"])
    for s in range(2):
        y = R.generator_forward(P, xn, geo, pqc=False)
        loss = 45.0 * R.multi_mel_loss(y, xc, [(2048, 300, 2048)], [R.hann(2048)], [mm], 1e-10, None)
        opt.zero_grad()
        loss.backward()
        tn = torch.nn.utils.clip_grad_norm_([P[k] for k in train], 1.0)
        opt.step()
        close(loss, g[f"loss.{s}"], rtol=1e-5)
        close(tn, g[f"gradnorm.{s}"], rtol=1e-4)
        for k in train:
            close(P[k], g[f"sd{s + 1}.{k}"], rtol=1e-5, atol=1e-7)


def test_stream_generator():
    """StreamGenerator (AudioDec.py:106-191): initial encode/decode on zeros, then
    six 600-sample chunks through encode -> quantize -> lookup -> decode, each
    conv carrying its pad_buffer (conv_layer.py:144-191)."""
    g = golden("stream")
    P = {k[3:]: T(v) for k, v in g.items() if k.startswith("sd.")}
    geo = R.generator_geometry(encode_channels=4, decode_channels=4)
    embeds = [P[f"quantizer.codebook.layers.{i}.embed"] for i in range(2)]
    S = {}
    z0 = R.stream_encode(P, S, torch.zeros(1, 1, 600), geo)
    zq0 = R.stream_lookup(R.stream_quantize(z0, embeds), embeds)
    close(zq0, g["init.zq"], rtol=1e-5, atol=1e-6)
    R.stream_decode(P, S, zq0, geo)
    x = T(g["x"])
    for c in range(6):
        z = R.stream_encode(P, S, x[:, :, 600 * c:600 * (c + 1)], geo)
        close(z, g[f"z.{c}"], rtol=1e-5, atol=1e-6)
        idx = R.stream_quantize(z, embeds)
        np.testing.assert_array_equal(idx.numpy(), g[f"idx.{c}"])
        zq = R.stream_lookup(idx, embeds)
        close(zq, g[f"zq.{c}"], rtol=1e-5, atol=1e-6)
        close(R.stream_decode(P, S, zq, geo), g[f"y.{c}"], rtol=1e-5, atol=1e-6)
    for k, v in g.items():
        if k.startswith("buf."):
            close(S[k[4:-len(".pad_buffer")]], v, rtol=1e-5, atol=1e-6)


def test_waveform_shape_loss():
    """losses/waveform_loss.py: multi-window and a window that leaves a tail."""
    g = golden("waveform")
    for tag, fn in (("multi", lambda a, b: R.multi_window_shape_loss(a, b)),
                    ("w160", lambda a, b: R.waveform_shape_loss(a, b, 160))):
        x = T(g["y_hat"]).requires_grad_(True)
        loss = fn(x, T(g["y"]))
        close(loss, g[f"{tag}.loss"], rtol=1e-6, atol=1e-8)
        loss.backward()
        close(x.grad, g[f"{tag}.grad"], rtol=1e-6, atol=1e-9)


# ---------------------------------------------------------------- GAN mode
D_PARAMS = dict(
    scales=3, scale_downsample_pooling_params={"kernel_size": 4, "stride": 2, "padding": 2},
    scale_discriminator_params={"in_channels": 1, "out_channels": 1, "kernel_sizes": [15, 41, 5, 3],
                                "channels": 16, "max_downsample_channels": 32, "max_groups": 16,
                                "downsample_scales": [4, 4, 4, 4, 1]},
    periods=[2, 3, 5, 7, 11],
    period_discriminator_params={"in_channels": 1, "out_channels": 1, "kernel_sizes": [5, 3], "channels": 4,
                                 "downsample_scales": [3, 3, 3, 3, 1], "max_downsample_channels": 32})


def gan_cotangent(shape, i, j):
    """Same deterministic cotangents as tests/golden/make_goldens.gan_cotangent."""
    return torch.randn(shape, generator=torch.Generator().manual_seed(1000 * i + j))


def _dparams(g, prefix="sd."):
    return {k[len(prefix):]: T(v).clone() for k, v in g.items() if k.startswith(prefix)}


def test_hifigan_discriminator():
    """HiFiGAN.Discriminator (HiFiGAN.py:308-395): all 8 x per-layer outputs and
    the gradients of sum(out * r) w.r.t. the input and every parameter."""
    g = golden("discriminator")
    P = _dparams(g)
    for v in P.values():
        v.requires_grad_(True)
    x = T(g["x"]).clone().requires_grad_(True)
    outs = R.hifigan_discriminator(P, x, **D_PARAMS)
    assert len(outs) == 8
    tot = 0.0
    for i, o in enumerate(outs):
        for j, t in enumerate(o):
            close(t, g[f"out.{i}.{j}"], rtol=1e-5, atol=1e-6)
            tot = tot + (t * gan_cotangent(t.shape, i, j)).sum()
    tot.backward()
    close(x.grad, g["grad_x"], rtol=1e-4, atol=1e-5)
    for k, v in P.items():
        close(v.grad, g["g." + k], rtol=1e-4, atol=1e-5)


def test_gan_losses():
    """adversarial_loss.py (mse + hinge, averaged or not) and feat_match_loss.py."""
    g = golden("discriminator")
    P = _dparams(g)
    with torch.no_grad():
        oy = R.hifigan_discriminator(P, T(g["y"]), **D_PARAMS)
        ox = R.hifigan_discriminator(P, T(g["x"]), **D_PARAMS)
    close(R.generator_adv_loss(ox, False), g["loss.gen_adv"], rtol=1e-6)
    close(R.generator_adv_loss(ox), g["loss.gen_adv_avg"], rtol=1e-6)
    close(R.generator_adv_loss(ox, loss_type="hinge"), g["loss.gen_adv_hinge"], rtol=1e-6)
    rl, fl = R.discriminator_adv_loss(ox, oy, False)
    close(rl, g["loss.dis_real"], rtol=1e-6)
    close(fl, g["loss.dis_fake"], rtol=1e-6)
    rl, fl = R.discriminator_adv_loss(ox, oy, loss_type="hinge")
    close(rl, g["loss.dis_real_hinge"], rtol=1e-6)
    close(fl, g["loss.dis_fake_hinge"], rtol=1e-6)
    close(R.feat_match_loss(ox, oy, False, False, False), g["loss.feat_match"], rtol=1e-6)
    close(R.feat_match_loss(ox, oy), g["loss.feat_match_default"], rtol=1e-6)
    close(R.feat_match_loss(ox, oy, include_final_outputs=True), g["loss.feat_match_final"], rtol=1e-6)
    x = T(g["x"]).clone().requires_grad_(True)
    oh = R.hifigan_discriminator(P, x, **D_PARAMS)
    (R.generator_adv_loss(oh, False) + 2.0 * R.feat_match_loss(oh, oy, False, False, False)).backward()
    close(x.grad, g["grad_x.gen_terms"], rtol=1e-4, atol=1e-7)


def test_gan_step():
    """Two GAN-mode train_denoise steps (:138-165, :213-263 with the discriminator
    enabled; vctk 48 kHz loss weights): generator 45*mel + adv (the waveform quirk,
    :147) + 2*feat-match, Adam(1e-4, (0.5, 0.9)); then the discriminator on the
    regenerated output, Adam(2e-4, (0.5, 0.9))."""
    g = golden("gan_step")
    Gp = _dparams(golden("generator_nopqc"))
    Dp = _dparams(golden("discriminator"))
    gm = golden("melmat")
    gtrain = [k for k in Gp if k.startswith(("encoder.", "decoder.conv_blocks", "decoder.conv2"))
              and not k.endswith("pad_buffer")]
    for k in gtrain:
        Gp[k].requires_grad_(True)
    for v in Dp.values():
        v.requires_grad_(True)
    og = torch.optim.Adam([Gp[k] for k in gtrain], lr=1e-4, betas=(0.5, 0.9), weight_decay=0.0)
    od = torch.optim.Adam(list(Dp.values()), lr=2e-4, betas=(0.5, 0.9), weight_decay=0.0)
    geo = R.generator_geometry(encode_channels=4, decode_channels=4)
    mm = T(gm["melmat.48k_fmax24000"])
    x, y = T(g["x_noisy"]), T(g["x_clean"])
    for s in range(2):
        pred = R.generator_forward(Gp, x, geo, pqc=False)
        mel = 45.0 * R.multi_mel_loss(pred, y, [(2048, 300, 2048)], [R.hann(2048)], [mm], 1e-10, None)
        p_ = R.hifigan_discriminator(Dp, pred, **D_PARAMS)
        with torch.no_grad():
            p = R.hifigan_discriminator(Dp, y, **D_PARAMS)
        adv = R.generator_adv_loss(pred, False)
        fm = 2.0 * R.feat_match_loss(p_, p)  # train_denoise.py:127: FeatureMatchLoss() defaults
        gen = mel + adv + fm
        og.zero_grad()
        od.zero_grad()
        gen.backward()
        og.step()
        with torch.no_grad():
            pred2 = R.generator_forward(Gp, x, geo, pqc=False)
        rl, fl = R.discriminator_adv_loss(R.hifigan_discriminator(Dp, pred2, **D_PARAMS),
                                          R.hifigan_discriminator(Dp, y, **D_PARAMS), False)
        dis = rl + fl
        od.zero_grad()
        dis.backward()
        od.step()
        for name, v in (("mel", mel), ("adv", adv), ("fm", fm), ("gen", gen), ("dis", dis)):
            close(v, g[f"{name}.{s}"], rtol=1e-5 if s == 0 else 1e-4)
        for k in gtrain:
            close(Gp[k], g[f"g_sd{s + 1}.{k}"], rtol=1e-5, atol=1e-7)
        for k, v in Dp.items():
            close(v, g[f"d_sd{s + 1}.{k}"], rtol=1e-5, atol=1e-7)


def test_denoise_trainer_step():
    """trainer/denoise.Trainer._train_step (:52-84) run by the reference class
    itself: PQC generator, codebook eval, lambda_vq * sum(vqloss) + 45 * mel
    (libritts-24k mel params), decoder/quantizer frozen, Adam(1e-4, (0.5, 0.9))."""
    g = golden("trainer_step")
    P = _dparams(g, "sd0.")
    train = [k for k in P if k.startswith(("encoder.", "projector.")) and k.endswith(("weight", "bias"))]
    for k in train:
        P[k].requires_grad_(True)
    opt = torch.optim.Adam([P[k] for k in train], lr=1e-4, betas=(0.5, 0.9), weight_decay=0.0)
    geo = R.generator_geometry(encode_channels=4, decode_channels=4)
    mm = T(golden("melmat")["melmat.24k_fmax12000"])
    xn, xc = T(g["x_noisy"]), T(g["x_clean"])
    for s in range(2):
        y, zq, z, vql, ppl = R.generator_forward(P, xn, geo, pqc=True, codebook_num=2)
        mel = 45.0 * R.multi_mel_loss(y, xc, [(2048, 300, 2048)], [R.hann(2048)], [mm], 1e-10, None)
        vq = vql.sum()
        loss = vq + mel
        opt.zero_grad()
        loss.backward()
        opt.step()
        close(mel, g[f"rec.{s}.train/mel_loss"], rtol=1e-5)
        close(vq, g[f"rec.{s}.train/train/vqloss"], rtol=1e-5)
        close(loss, g[f"rec.{s}.train/generator_loss"], rtol=1e-5)
        for i in range(2):
            close(ppl[i], g[f"rec.{s}.train/train/ppl_{i}"], rtol=1e-5)
        for k in train:
            close(P[k], g[f"sd{s + 1}.{k}"], rtol=1e-5, atol=1e-7)


# ---- layer forms outside the shipped causal configs (tests/golden/general_conv.npz) ----

def _general_case(g, name, fn):
    x = T(g[f"{name}.x"]).requires_grad_(True)
    w = T(g[f"{name}.w"]).requires_grad_(True)
    b = T(g[f"{name}.b"]).requires_grad_(True) if f"{name}.b" in g else None
    y = fn(x, w, b)
    close(y, g[f"{name}.y"], rtol=1e-5, atol=1e-5)
    y.backward(T(g[f"{name}.gy"]))
    close(x.grad, g[f"{name}.gx"], rtol=1e-5, atol=1e-5)
    close(w.grad, g[f"{name}.gw"], rtol=1e-5, atol=1e-4)
    if b is not None:
        close(b.grad, g[f"{name}.gb"], rtol=1e-5, atol=1e-4)


def test_general_conv_layers():
    """NonCausalConv1d / NonCausalConvTranspose1d with any stride, padding,
    dilation, groups; grouped and odd-stride CausalConv1d; CausalConvTranspose1d
    with k != 2s (layers/conv_layer.py:26-191) against the reference's own layers."""
    from golden.make_goldens import GENERAL_CAUSAL, GENERAL_CAUSALT, GENERAL_CONV, GENERAL_CONVT
    g = golden("general_conv")
    for name, ci, co, k, s, p, dl, gr, b, t in GENERAL_CONV:
        _general_case(g, name, lambda x, w, bb: R.noncausal_conv1d(x, w, bb, s, p, dl, gr))
    for name, ci, co, k, s, p, op, gr, b, t in GENERAL_CONVT:
        _general_case(g, name, lambda x, w, bb: R.noncausal_conv_transpose1d(x, w, bb, s, p, op, gr))
    for name, ci, co, k, s, dl, gr, b, t in GENERAL_CAUSAL:
        _general_case(g, name, lambda x, w, bb: R.grouped_causal_conv1d(x, w, bb, s, dl, gr))
    for name, ci, co, k, s, t in GENERAL_CAUSALT:
        _general_case(g, name, lambda x, w, bb: R.causal_conv_transpose1d(x, w, bb, s))


@pytest.mark.parametrize("tag", ["pqc", "nopqc"])
def test_noncausal_generator(tag):
    """Generator(mode='noncausal') (encoder.py:38-57, decoder.py:38-57, residual_unit.py:20-46)."""
    g = golden(f"generator_noncausal_{tag}")
    gm = golden("melmat")
    P = {k[3:]: T(v) for k, v in g.items() if k.startswith("sd.")}
    for k, v in P.items():
        if v.dtype == torch.float32 and not k.endswith(("pad_buffer", "embed", "cluster_size", "embed_avg")):
            v.requires_grad_(True)
    geo = R.generator_geometry(encode_channels=4, decode_channels=4)
    xn, xc = T(g["x_noisy"]), T(g["x_clean"])
    mm = T(gm["melmat.24k_fmax24000"])
    mel = lambda a, b: R.multi_mel_loss(a, b, [(2048, 300, 2048)], [R.hann(2048)], [mm], 1e-10, None)
    if tag == "pqc":
        y, zq, z, vql, ppl = R.generator_forward(P, xn, geo, pqc=True, codebook_num=2, mode="noncausal")
        close(z, g["z"], rtol=1e-5, atol=1e-6)
        close(zq, g["zq"], rtol=1e-5, atol=1e-6)
        close(vql, g["vqloss"], rtol=1e-5, atol=1e-7)
        loss = 45.0 * mel(y, xc) + vql.sum()
    else:
        y = R.generator_forward(P, xn, geo, pqc=False, mode="noncausal")
        loss = 45.0 * mel(y, xc)
    close(y, g["y"], rtol=1e-5, atol=1e-6)
    close(loss, g["loss"], rtol=1e-5)
    loss.backward()
    for k, v in g.items():
        if k.startswith("g."):
            close(P[k[2:]].grad, v, rtol=1e-4, atol=1e-6)


def test_spectral_norm_period_discriminator():
    """discriminator.py:99-157 with use_spectral_norm: one training-mode power
    iteration per call (torch.nn.utils.spectral_norm), outputs, input and
    weight_orig gradients, and the updated u / v buffers."""
    g = golden("spectral_norm")
    sd0 = {k[4:]: T(v) for k, v in g.items() if k.startswith("sd0.")}
    P = {f"d.{k}": v.clone().requires_grad_(k.endswith(("weight_orig", "bias"))) for k, v in sd0.items()}
    plan = R.period_discriminator_plan(channels=4, max_downsample_channels=32)
    for key in [k for k in sd0 if k.endswith("weight_orig")]:
        m = key[:-len(".weight_orig")]
        _, u, v = R.spectral_norm_weight(sd0[key], sd0[m + ".weight_u"], sd0[m + ".weight_v"])
        close(u, g[f"sd1.{m}.weight_u"], rtol=1e-5, atol=1e-7)
        close(v, g[f"sd1.{m}.weight_v"], rtol=1e-5, atol=1e-7)
    x = T(g["x"]).requires_grad_(True)
    outs = R.period_discriminator(P, "d", x, 3, plan)
    for j, o in enumerate(outs):
        close(o, g[f"out.{j}"], rtol=1e-5, atol=1e-6)
    sum((o * R_cot(o.shape, j)).sum() for j, o in enumerate(outs)).backward()
    close(x.grad, g["grad_x"], rtol=1e-4, atol=1e-6)
    for k, v in g.items():
        if k.startswith("g."):
            close(P["d." + k[2:]].grad, v, rtol=1e-4, atol=1e-6)


def R_cot(shape, j):
    """tests/golden/make_goldens.gan_cotangent(shape, 0, j)."""
    return torch.randn(shape, generator=torch.Generator().manual_seed(j))


def test_conv1d_bn_projector_generator():
    """Generator(projector='conv1d_bn') (projector.py:40-44): BatchNorm1d in
    training mode (outputs, gradients, running statistics), then evaluation."""
    g = golden("generator_bn")
    gm = golden("melmat")
    P = {k[3:]: T(v) for k, v in g.items() if k.startswith("sd.")}
    for k, v in P.items():
        if v.dtype == torch.float32 and not k.endswith(("pad_buffer", "embed", "cluster_size", "embed_avg",
                                                         "running_mean", "running_var")):
            v.requires_grad_(True)
    geo = R.generator_geometry(encode_channels=4, decode_channels=4)
    xn, xc = T(g["x_noisy"]), T(g["x_clean"])
    mm = T(gm["melmat.24k_fmax24000"])
    y, zq, z, vql, ppl = R.generator_forward(P, xn, geo, pqc=True, codebook_num=2)
    close(z, g["z"], rtol=1e-5, atol=1e-5)
    close(y, g["y"], rtol=1e-5, atol=1e-5)  # BN divides by the batch std
    loss = 45.0 * R.multi_mel_loss(y, xc, [(2048, 300, 2048)], [R.hann(2048)], [mm], 1e-10, None) + vql.sum()
    close(loss, g["loss"], rtol=1e-5)
    loss.backward()
    for k, v in g.items():
        if k.startswith("g."):
            close(P[k[2:]].grad, v, rtol=1e-4, atol=1e-5)
    for k in ("running_mean", "running_var"):
        close(P[f"projector.project.1.{k}"], g[f"sd1.projector.project.1.{k}"], rtol=1e-5, atol=1e-7)
    with torch.no_grad():
        y, zq, z, vql, ppl = R.generator_forward(P, xn, geo, pqc=True, codebook_num=2, training=False)
    close(z, g["eval.z"], rtol=1e-5, atol=1e-5)
    close(y, g["eval.y"], rtol=1e-5, atol=1e-5)
