"""Generate golden vectors by importing the reference (build container only).

Run:  python tests/golden/make_goldens.py  [--ref /root/reference]

This imports s194584/dl-speech-enhancement from ``/root/reference`` (read-only,
never copied, never shipped) and records inputs/outputs of the hot-path
modules as small ``.npz`` fixtures under ``tests/golden/``.  Those fixtures pin
the CPU oracle (``oracle/``) and, through it, the HIP path.

Third-party pieces absent from this image and how they are handled:
* librosa 0.8.1 (``losses/mel_loss.py:14``) — injected as a stub module whose
  ``filters.mel`` is the restatement in ``oracle/melfilters.py``.
* torchaudio / soundfile (dataloader package init) — ``dataloader/data_utils.py``
  and ``collater.py`` are loaded by file path with a stub package.
* torchmetrics (SNR), clearml — not needed: the step glue of
  ``train_denoise.py:213-263`` is restated below from its source text.
* tensorboardX (``trainer/trainerGAN.py:20``) — stub ``SummaryWriter`` (no-op)
  so the reference ``trainer/denoise.Trainer`` itself runs (``--only trainer``).
* torchaudio (``models/vocoder/modules/discriminator.py:23`` imports
  ``functional.spectrogram``, used only by the UnivNet discriminator) — stub
  module, so the HiFiGAN discriminator itself runs (``--only gan``).
"""
import argparse
import importlib.util
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from oracle import melfilters  # noqa: E402


def _install_stubs(ref):
    lib = types.ModuleType("librosa")
    lib.filters = types.SimpleNamespace(mel=melfilters.mel)
    sys.modules["librosa"] = lib
    sys.path.insert(0, ref)
    # dataloader package init pulls torchaudio/soundfile: load the two files we need by path.
    pkg = types.ModuleType("dataloader")
    pkg.__path__ = [os.path.join(ref, "dataloader")]
    sys.modules["dataloader"] = pkg
    col = _load("dataloader.collater", os.path.join(ref, "dataloader", "collater.py"))
    pkg.CollaterAudio = col.CollaterAudio
    pkg.CollaterAudioPair = col.CollaterAudioPair
    du = _load("dataloader.data_utils", os.path.join(ref, "dataloader", "data_utils.py"))
    return du


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def _audio(ref):
    """Real speech/noise from reference notebook_files (48k int16 clean, 24k f32 noise)."""
    from scipy.io import wavfile
    from scipy.signal import resample_poly
    import warnings
    warnings.filterwarnings("ignore")
    clean = []
    noise = []
    for i in (1, 2):
        sr, d = wavfile.read(os.path.join(ref, "notebook_files", f"clean{i}.wav"))
        x = d.astype(np.float64) / 32768.0
        clean.append(resample_poly(x, 1, sr // 24000).astype(np.float32))
        sr, d = wavfile.read(os.path.join(ref, "notebook_files", f"noise{i}.wav"))
        n = d.astype(np.float32)
        if sr != 24000:
            n = resample_poly(n.astype(np.float64), 24000, sr).astype(np.float32)
        noise.append(n)
    return clean, noise


def _np(t):
    return t.detach().cpu().numpy().copy()  # never alias live parameters


def _sd(module, prefix="sd."):
    return {prefix + k: _np(v) for k, v in module.state_dict().items()}


def _params(module, prefix):
    return {prefix + k: _np(p) for k, p in module.named_parameters()}


def _grads(module, prefix="g."):
    return {prefix + k: _np(p.grad) for k, p in module.named_parameters() if p.grad is not None}


def make_stream(pqc_mod, clean, noise, gp, out):
    """StreamGenerator at reduced width: initial_encoder/decoder on zeros, then six
    600-sample chunks (2 latent frames each) through encode -> quantize -> lookup ->
    decode, recording every intermediate and the final pad_buffers."""
    torch.manual_seed(93)
    G = pqc_mod.StreamGenerator(**gp)
    G.eval()
    d = _sd(G)
    x = torch.from_numpy(clean[0][:3600] + 0.1 * noise[0][:3600]).float().view(1, 1, -1)
    d["x"] = _np(x)
    with torch.no_grad():
        zq0 = G.initial_encoder(600, "cpu")
        G.initial_decoder(zq0)
        d["init.zq"] = _np(zq0)
        for c in range(6):
            xc = x[:, :, 600 * c:600 * (c + 1)]
            z = G.encode(xc)
            idx = G.quantize(z)
            zq = G.lookup(idx)
            y = G.decode(zq)
            d.update({f"z.{c}": _np(z), f"idx.{c}": _np(idx), f"zq.{c}": _np(zq), f"y.{c}": _np(y)})
    d.update({"buf." + k: _np(v) for k, v in G.state_dict().items() if k.endswith("pad_buffer")})
    np.savez_compressed(os.path.join(out, "stream.npz"), **d)


def make_waveform(ref, clean, noise, out):
    """losses/waveform_loss.py: MultiWindowShapeLoss (default windows) and a
    single WaveformShapeLoss(160) whose window does not divide T."""
    wl = _load("ref_waveform_loss", os.path.join(ref, "losses", "waveform_loss.py"))
    T = 4810
    y = torch.from_numpy(np.stack([clean[0][:T], clean[1][:T]])).unsqueeze(1)
    yh = torch.from_numpy(np.stack([clean[0][:T] + 0.2 * noise[0][:T],
                                    clean[1][:T] + 0.2 * noise[1][:T]]).astype(np.float32)).unsqueeze(1)
    d = {"y": _np(y), "y_hat": _np(yh)}
    for tag, mod in (("multi", wl.MultiWindowShapeLoss()), ("w160", wl.WaveformShapeLoss(160))):
        x = yh.clone().requires_grad_(True)
        loss = mod(x, y)
        loss.backward()
        d[f"{tag}.loss"] = _np(loss)
        d[f"{tag}.grad"] = _np(x.grad)
    np.savez_compressed(os.path.join(out, "waveform.npz"), **d)


def _install_trainer_stubs():
    tbx = types.ModuleType("tensorboardX")

    class SummaryWriter:  # no-op stand-in (logging only)
        def __init__(self, *a, **k):
            pass

        def add_scalar(self, *a, **k):
            pass

    tbx.SummaryWriter = SummaryWriter
    sys.modules["tensorboardX"] = tbx
    ta = types.ModuleType("torchaudio")
    ta.functional = types.SimpleNamespace(spectrogram=None)
    sys.modules["torchaudio"] = ta
    sys.modules["torchaudio.functional"] = ta.functional


# reduced-width HiFiGAN discriminator: the vctk 48 kHz structure
# (config/denoise/symAD_vctk_48000_hop300.yaml:49-82) at 1/8 .. 1/32 the channels
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
    """Deterministic cotangent for output (i, j) (regenerated by the tests, not stored)."""
    return torch.randn(shape, generator=torch.Generator().manual_seed(1000 * i + j))


def _flat_outs(outs, prefix):
    d = {}
    for i, o in enumerate(outs):
        for j, t in enumerate(o):
            d[f"{prefix}.{i}.{j}"] = _np(t)
    return d


def make_gan(ref, clean, noise, out):
    """HiFiGAN MSD+MPD discriminator (models/vocoder/HiFiGAN.py:308-395), the
    adversarial / feature-matching losses (losses/adversarial_loss.py,
    feat_match_loss.py) and two GAN-mode train_denoise steps (:138-165, :213-263,
    restated from the source text; discriminator enabled) at reduced width."""
    _install_trainer_stubs()
    hifi = importlib.import_module("models.vocoder.HiFiGAN")
    adv = _load("ref_adversarial_loss", os.path.join(ref, "losses", "adversarial_loss.py"))
    fm = _load("ref_feat_match_loss", os.path.join(ref, "losses", "feat_match_loss.py"))
    mel_mod = _load("ref_mel_loss", os.path.join(ref, "losses", "mel_loss.py"))
    npqc_mod = importlib.import_module("models.autoencoder_without_PQC.AudioDec")
    T = 1200  # 25 ms at 48 kHz: MPD reflect-pads for periods 7 and 11 (1200 % p != 0)
    torch.manual_seed(93)
    D = hifi.Discriminator(**D_PARAMS)
    d = _sd(D)
    x = torch.from_numpy(np.stack([clean[0][:T] + 0.1 * noise[0][:T],
                                   clean[1][:T] + 0.1 * noise[1][:T]]).astype(np.float32)).unsqueeze(1)
    y = torch.from_numpy(np.stack([clean[0][:T], clean[1][:T]])).unsqueeze(1)
    d["x"], d["y"] = _np(x), _np(y)
    xg = x.clone().requires_grad_(True)
    outs = D(xg)
    d.update(_flat_outs(outs, "out"))
    r = [[gan_cotangent(t.shape, i, j) for j, t in enumerate(o)] for i, o in enumerate(outs)]
    sum((t * rr).sum() for o, ro in zip(outs, r) for t, rr in zip(o, ro)).backward()
    d["grad_x"] = _np(xg.grad)
    d.update(_grads(D))
    with torch.no_grad():
        outs_y = D(y)
        outs_x = D(x)
    gal = adv.GeneratorAdversarialLoss(average_by_discriminators=False)
    dal = adv.DiscriminatorAdversarialLoss(average_by_discriminators=False)
    fml = fm.FeatureMatchLoss(average_by_discriminators=False, average_by_layers=False,
                              include_final_outputs=False)
    d["loss.gen_adv"] = _np(gal(outs_x))
    d["loss.gen_adv_avg"] = _np(adv.GeneratorAdversarialLoss()(outs_x))
    d["loss.gen_adv_hinge"] = _np(adv.GeneratorAdversarialLoss(loss_type="hinge")(outs_x))
    rl, fl = dal(outs_x, outs_y)
    d["loss.dis_real"], d["loss.dis_fake"] = _np(rl), _np(fl)
    rl, fl = adv.DiscriminatorAdversarialLoss(loss_type="hinge")(outs_x, outs_y)
    d["loss.dis_real_hinge"], d["loss.dis_fake_hinge"] = _np(rl), _np(fl)
    d["loss.feat_match"] = _np(fml(outs_x, outs_y))
    d["loss.feat_match_default"] = _np(fm.FeatureMatchLoss()(outs_x, outs_y))
    d["loss.feat_match_final"] = _np(fm.FeatureMatchLoss(include_final_outputs=True)(outs_x, outs_y))
    # gradients of the two GAN loss terms w.r.t. the fake input
    xg = x.clone().requires_grad_(True)
    o_hat = D(xg)
    (gal(o_hat) + 2.0 * fml(o_hat, outs_y)).backward()
    d["grad_x.gen_terms"] = _np(xg.grad)
    np.savez_compressed(os.path.join(out, "discriminator.npz"), **d)

    # ---- two GAN-mode train_denoise steps (discriminator enabled) ----
    gp = dict(encode_channels=4, decode_channels=4, code_dim=64, codebook_num=2, codebook_size=64)
    p48 = dict(fs=48000, fft_sizes=[2048], hop_sizes=[300], win_lengths=[None], window="hann_window",
               num_mels=80, fmin=0, fmax=24000, log_base=None)
    # initial weights = generator_nopqc.npz sd (seed 93) and discriminator.npz sd (seed 93): not stored again
    torch.manual_seed(93)
    G = npqc_mod.Generator(**gp)
    torch.manual_seed(93)
    D = hifi.Discriminator(**D_PARAMS)
    mel = mel_mod.MultiMelSpectrogramLoss(**p48)
    og = torch.optim.Adam(G.parameters(), lr=1e-4, betas=(0.5, 0.9), weight_decay=0.0)
    od = torch.optim.Adam(D.parameters(), lr=2e-4, betas=(0.5, 0.9), weight_decay=0.0)
    g = {"x_noisy": _np(x), "x_clean": _np(y)}
    lam_mel, lam_adv, lam_fm = 45.0, 1.0, 2.0
    fm_step = fm.FeatureMatchLoss()
    for step in range(2):
        G.train()
        D.train()
        pred = G(x)
        mel_loss = lam_mel * mel(pred, y)
        p_ = D(pred)
        with torch.no_grad():
            p = D(y)
        adv_loss = lam_adv * gal(pred)  # reference quirk (:147): the waveform, not p_
        feat_loss = lam_fm * fm_step(p_, p)  # train_denoise.py:127 builds FeatureMatchLoss() (defaults)
        gen_loss = mel_loss + adv_loss + feat_loss
        og.zero_grad()
        gen_loss.backward()
        og.step()
        with torch.no_grad():
            pred2 = G(x)
        p = D(y)
        p_ = D(pred2.detach())
        rl, fl = dal(p_, p)
        dis_loss = (rl + fl) * lam_adv
        od.zero_grad()
        dis_loss.backward()
        od.step()
        g.update({f"mel.{step}": _np(mel_loss), f"adv.{step}": _np(adv_loss), f"fm.{step}": _np(feat_loss),
                  f"gen.{step}": _np(gen_loss), f"dis.{step}": _np(dis_loss)})
        g.update(_params(G, f"g_sd{step + 1}."))
        g.update(_params(D, f"d_sd{step + 1}."))
    np.savez_compressed(os.path.join(out, "gan_step.npz"), **g)


def make_trainer(ref, clean, noise, out):
    """trainer/denoise.Trainer._train_step (the reference class itself, :52-84)
    on the reduced-width PQC generator for two steps, then its save_checkpoint
    (trainerGAN.py:95-121) with a reduced HiFiGAN discriminator."""
    _install_trainer_stubs()
    sys.modules.pop("trainer", None)
    den = importlib.import_module("trainer.denoise")
    hifi = importlib.import_module("models.vocoder.HiFiGAN")
    mel_mod = _load("ref_mel_loss", os.path.join(ref, "losses", "mel_loss.py"))
    pqc_mod = importlib.import_module("models.autoencoder.AudioDec")
    gp = dict(encode_channels=4, decode_channels=4, code_dim=64, codebook_num=2, codebook_size=64)
    p24 = dict(fs=24000, fft_sizes=[2048], hop_sizes=[300], win_lengths=[2048], window="hann_window",
               num_mels=80, fmin=0, fmax=12000, log_base=None)
    T = 2400
    xn = torch.from_numpy(np.stack([clean[0][:T] + 0.1 * noise[0][:T],
                                    clean[1][:T] + 0.1 * noise[1][:T]]).astype(np.float32)).unsqueeze(1)
    xc = torch.from_numpy(np.stack([clean[0][:T], clean[1][:T]])).unsqueeze(1)
    torch.manual_seed(95)
    G = pqc_mod.Generator(**gp)
    D = hifi.Discriminator(**D_PARAMS)
    cfg = {"outdir": None, "train_max_steps": 10, "use_mel_loss": True, "use_stft_loss": False,
           "use_shape_loss": False, "lambda_mel_loss": 45.0, "lambda_vq_loss": 1.0, "generator_grad_norm": -1}
    og = torch.optim.Adam(G.parameters(), lr=1e-4, betas=(0.5, 0.9), weight_decay=0.0)
    od = torch.optim.Adam(D.parameters(), lr=2e-4, betas=(0.5, 0.9), weight_decay=0.0)
    sg = torch.optim.lr_scheduler.StepLR(og, step_size=200000, gamma=1.0)
    sd = torch.optim.lr_scheduler.MultiStepLR(od, milestones=[200000, 400000], gamma=0.5)
    d = {"x_noisy": _np(xn), "x_clean": _np(xc)}
    d.update(_sd(G, "sd0."))
    tr = den.Trainer(steps=0, epochs=0, data_loader={}, model={"generator": G, "discriminator": D},
                     criterion={"mel": mel_mod.MultiMelSpectrogramLoss(**p24)},
                     optimizer={"generator": og, "discriminator": od},
                     scheduler={"generator": sg, "discriminator": sd}, config=cfg)
    tr.tqdm = types.SimpleNamespace(update=lambda n=1: None)
    for step in range(2):
        tr._train_step((xn, xc))
        for k, v in tr.total_train_loss.items():
            d[f"rec.{step}.{k}"] = np.array(v, dtype=np.float64)
        tr.total_train_loss.clear()
        d.update({f"sd{step + 1}.{k}": _np(p) for k, p in G.named_parameters() if p.requires_grad})
    tr.save_checkpoint(os.path.join(out, "trainer_ckpt.pt"))
    np.savez_compressed(os.path.join(out, "trainer_step.npz"), **d)


# (name, Cin, Cout, k, stride, padding, dilation, groups, bias, T) of NonCausalConv1d
GENERAL_CONV = [
    ("nc_same", 8, 8, 7, 1, -1, 3, 1, False, 100),
    ("nc_down3", 8, 16, 6, 3, -1, 1, 1, True, 240),     # noncausal EncoderBlock conv (encoder.py:50-57)
    ("nc_s2_p0", 6, 10, 5, 2, 0, 1, 1, True, 101),
    ("nc_grp", 8, 12, 5, 1, 2, 2, 4, True, 90),
    ("nc_grp_s4", 16, 16, 41, 4, 20, 1, 4, True, 200),  # the MSD's grouped k41 layer shape, 41 taps
    ("nc_bigpad", 4, 6, 3, 1, 5, 1, 1, True, 50),
]
# (name, Cin, Cout, k, stride, padding, output_padding, groups, bias, T) of NonCausalConvTranspose1d
GENERAL_CONVT = [
    ("nct_up5", 16, 8, 10, 5, -1, -1, 1, True, 20),    # noncausal DecoderBlock deconv (decoder.py:47-54)
    ("nct_up4", 12, 8, 8, 4, -1, -1, 1, True, 25),
    ("nct_grp", 8, 12, 5, 3, 1, 2, 4, True, 30),
    ("nct_k3s1", 6, 4, 3, 1, 0, 0, 1, False, 40),
]
# grouped / odd-stride CausalConv1d: (name, Cin, Cout, k, stride, dilation, groups, bias, T)
GENERAL_CAUSAL = [
    ("c_grp", 8, 8, 7, 1, 2, 2, True, 100),
    ("c_s3k4", 6, 8, 4, 3, 1, 1, True, 100),
]
# CausalConvTranspose1d with k != 2s: (name, Cin, Cout, k, stride, T)
GENERAL_CAUSALT = [("ct_k3s2", 8, 4, 3, 2, 30), ("ct_k7s3", 6, 6, 7, 3, 20)]


def _record(d, name, m, conv, xin, cfg):
    yo = m(xin)
    gy = torch.randn_like(yo)
    yo.backward(gy)
    d[f"{name}.cfg"] = np.array(cfg)
    d[f"{name}.x"], d[f"{name}.w"] = _np(xin), _np(conv.weight)
    d[f"{name}.y"], d[f"{name}.gy"] = _np(yo), _np(gy)
    d[f"{name}.gx"], d[f"{name}.gw"] = _np(xin.grad), _np(conv.weight.grad)
    if conv.bias is not None:
        d[f"{name}.b"], d[f"{name}.gb"] = _np(conv.bias), _np(conv.bias.grad)


def make_general(ref, clean, noise, out):
    """Layer forms outside the shipped causal configs (layers/conv_layer.py:26-191
    with any stride / padding / dilation / groups), the noncausal AudioDec
    generators (mode='noncausal', encoder.py:38-57, decoder.py:38-57) and a
    spectral-normalised period discriminator (discriminator.py:99-157)."""
    conv_mod = importlib.import_module("layers.conv_layer")
    torch.manual_seed(7)
    d = {}
    for name, ci, co, k, s, p, dl, g, b, t in GENERAL_CONV:
        m = conv_mod.NonCausalConv1d(ci, co, k, stride=s, padding=p, dilation=dl, groups=g, bias=b)
        _record(d, name, m, m.conv, torch.randn(2, ci, t, requires_grad=True), [ci, co, k, s, p, dl, g, int(b), t])
    for name, ci, co, k, s, p, op, g, b, t in GENERAL_CONVT:
        m = conv_mod.NonCausalConvTranspose1d(ci, co, k, s, padding=p, output_padding=op, groups=g, bias=b)
        _record(d, name, m, m.deconv, torch.randn(2, ci, t, requires_grad=True), [ci, co, k, s, p, op, g, int(b), t])
    for name, ci, co, k, s, dl, g, b, t in GENERAL_CAUSAL:
        m = conv_mod.CausalConv1d(ci, co, k, stride=s, dilation=dl, groups=g, bias=b)
        _record(d, name, m, m.conv, torch.randn(2, ci, t, requires_grad=True), [ci, co, k, s, dl, g, int(b), t])
    for name, ci, co, k, s, t in GENERAL_CAUSALT:
        m = conv_mod.CausalConvTranspose1d(ci, co, k, s)
        _record(d, name, m, m.deconv, torch.randn(2, ci, t, requires_grad=True), [ci, co, k, s, t])
    np.savez_compressed(os.path.join(out, "general_conv.npz"), **d)

    # noncausal generators (reduced width), as the causal generator_{pqc,nopqc} fixtures
    mel_mod = _load("ref_mel_loss", os.path.join(ref, "losses", "mel_loss.py"))
    mel = mel_mod.MultiMelSpectrogramLoss(fs=24000, fft_sizes=[2048], hop_sizes=[300], win_lengths=[None],
                                          window="hann_window", num_mels=80, fmin=0, fmax=24000, log_base=None)
    gp = dict(encode_channels=4, decode_channels=4, code_dim=64, codebook_num=2, codebook_size=64)
    T = 2400
    xn = torch.from_numpy(np.stack([clean[0][:T] + 0.1 * noise[0][:T],
                                    clean[1][:T] + 0.1 * noise[1][:T]]).astype(np.float32)).unsqueeze(1)
    xc = torch.from_numpy(np.stack([clean[0][:T], clean[1][:T]])).unsqueeze(1)
    for tag, mod in (("pqc", "models.autoencoder.AudioDec"), ("nopqc", "models.autoencoder_without_PQC.AudioDec")):
        torch.manual_seed(93)
        G = importlib.import_module(mod).Generator(mode="noncausal", **gp)
        d = {"x_noisy": _np(xn), "x_clean": _np(xc)}
        d.update(_sd(G))
        if tag == "pqc":
            G.quantizer.codebook.eval()
            y, zq, z, vql, ppl = G(xn)
            loss = 45.0 * mel(y, xc) + vql.sum()
            d.update({"y": _np(y), "zq": _np(zq), "z": _np(z), "vqloss": _np(vql), "ppl": _np(ppl)})
        else:
            y = G(xn)
            loss = 45.0 * mel(y, xc)
            d["y"] = _np(y)
        loss.backward()
        d["loss"] = _np(loss)
        d.update(_grads(G))
        np.savez_compressed(os.path.join(out, f"generator_noncausal_{tag}.npz"), **d)

    # projector model='conv1d_bn' (projector.py:40-44): BatchNorm1d in training mode, then evaluation
    torch.manual_seed(93)
    G = importlib.import_module("models.autoencoder.AudioDec").Generator(projector="conv1d_bn", **gp)
    G.quantizer.codebook.eval()
    d = {"x_noisy": _np(xn), "x_clean": _np(xc)}
    d.update(_sd(G))
    y, zq, z, vql, ppl = G(xn)
    loss = 45.0 * mel(y, xc) + vql.sum()
    d.update({"y": _np(y), "zq": _np(zq), "z": _np(z), "vqloss": _np(vql), "loss": _np(loss)})
    loss.backward()
    d.update(_grads(G))
    d.update(_sd(G, "sd1."))
    G.eval()
    with torch.no_grad():
        y, zq, z, vql, ppl = G(xn)
    d.update({"eval.y": _np(y), "eval.z": _np(z)})
    np.savez_compressed(os.path.join(out, "generator_bn.npz"), **d)

    # spectral-normalised period discriminator, training mode (one power iteration per call)
    _install_trainer_stubs()
    disc = importlib.import_module("models.vocoder.modules.discriminator")
    torch.manual_seed(11)
    D = disc.HiFiGANPeriodDiscriminator(period=3, channels=4, max_downsample_channels=32,
                                        use_weight_norm=False, use_spectral_norm=True)
    d = _sd(D, "sd0.")
    x = torch.from_numpy(np.stack([clean[0][:600], clean[1][:600]])).unsqueeze(1).requires_grad_(True)
    d["x"] = _np(x)
    outs = D(x)
    d.update({f"out.{j}": _np(t) for j, t in enumerate(outs)})
    sum((t * gan_cotangent(t.shape, 0, j)).sum() for j, t in enumerate(outs)).backward()
    d["grad_x"] = _np(x.grad)
    d.update(_grads(D))
    d.update(_sd(D, "sd1."))
    np.savez_compressed(os.path.join(out, "spectral_norm.npz"), **d)


def make(ref, out, only=None):
    du = _install_stubs(ref)
    stft_mod = _load("ref_stft_loss", os.path.join(ref, "losses", "stft_loss.py"))
    mel_mod = _load("ref_mel_loss", os.path.join(ref, "losses", "mel_loss.py"))
    conv_mod = importlib.import_module("layers.conv_layer")
    vq_mod = importlib.import_module("layers.vq_module")
    pqc_mod = importlib.import_module("models.autoencoder.AudioDec")
    npqc_mod = importlib.import_module("models.autoencoder_without_PQC.AudioDec")

    clean, noise = _audio(ref)
    os.makedirs(out, exist_ok=True)
    if only == "stream":
        gp = dict(encode_channels=4, decode_channels=4, code_dim=64, codebook_num=2, codebook_size=64)
        return make_stream(pqc_mod, clean, noise, gp, out)
    if only == "waveform":
        return make_waveform(ref, clean, noise, out)
    if only == "gan":
        return make_gan(ref, clean, noise, out)
    if only == "general":
        return make_general(ref, clean, noise, out)
    if only == "trainer":
        return make_trainer(ref, clean, noise, out)
    torch.manual_seed(93)

    # ---------------- melmat (losses/mel_loss.py:54-61) ----------------
    cfgs = {
        "24k_fmax24000": dict(fs=24000, fft_size=2048, hop_size=300, win_length=None, num_mels=80, fmin=0, fmax=24000, log_base=None),
        "24k_fmax12000": dict(fs=24000, fft_size=2048, hop_size=300, win_length=2048, num_mels=80, fmin=0, fmax=12000, log_base=None),
        "48k_fmax24000": dict(fs=48000, fft_size=2048, hop_size=300, win_length=None, num_mels=80, fmin=0, fmax=24000, log_base=None),
        "default": dict(),
    }
    d = {}
    for k, c in cfgs.items():
        m = mel_mod.MelSpectrogram(**c)
        d[f"melmat.{k}"] = _np(m.melmat)
        d[f"window.{k}"] = _np(m.window)
    np.savez_compressed(os.path.join(out, "melmat.npz"), **d)

    # ---------------- stft magnitude + losses (losses/stft_loss.py) ----------------
    T = 12000
    x = torch.from_numpy(np.stack([clean[0][4000:4000 + T], clean[1][8000:8000 + T]]))
    y = torch.from_numpy(np.stack([clean[0][4000:4000 + T] + 0.05 * noise[0][:T],
                                   clean[1][8000:8000 + T] + 0.05 * noise[1][:T]]).astype(np.float32))
    d = {"x": _np(x), "y": _np(y)}
    res = [(1024, 120, 600), (2048, 240, 1200), (512, 50, 240)]
    for n, h, w in res:
        win = torch.hann_window(w)
        d[f"mag.{n}"] = _np(stft_mod.stft(x, n, h, w, win))
        sl = stft_mod.STFTLoss(n, h, w)
        sc, mg = sl(x, y)
        d[f"sc.{n}"] = _np(sc)
        d[f"logmag.{n}"] = _np(mg)
    xg = x.clone().requires_grad_(True)
    mr = stft_mod.MultiResolutionSTFTLoss()
    sc, mg = mr(xg.unsqueeze(1), y.unsqueeze(1))
    (sc + mg).backward()
    d["mr.sc"] = _np(sc)
    d["mr.mag"] = _np(mg)
    d["mr.grad_x"] = _np(xg.grad)
    # edge case: shortest legal signal for n_fft 2048 (reflect pad needs T > n_fft/2)
    xs = torch.from_numpy(clean[0][:1025].copy()).unsqueeze(0)
    d["short.x"] = _np(xs)
    d["short.mag.2048"] = _np(stft_mod.stft(xs, 2048, 240, 1200, torch.hann_window(1200)))
    np.savez_compressed(os.path.join(out, "stft.npz"), **d)

    # ---------------- mel loss (losses/mel_loss.py) ----------------
    T = 24000
    yh = torch.from_numpy(np.stack([clean[0][:T] * 0.7 + 0.02 * noise[0][:T],
                                    clean[1][:T] * 0.7 + 0.02 * noise[1][:T]]).astype(np.float32)).unsqueeze(1)
    yt = torch.from_numpy(np.stack([clean[0][:T], clean[1][:T]])).unsqueeze(1)
    d = {"y_hat": _np(yh), "y": _np(yt)}
    p24 = dict(fs=24000, fft_sizes=[2048], hop_sizes=[300], win_lengths=[None], window="hann_window",
               num_mels=80, fmin=0, fmax=24000, log_base=None)
    ml = mel_mod.MultiMelSpectrogramLoss(**p24)
    d["mel24.y_hat"] = _np(ml.mel_transfers[0](yh))
    g = yh.clone().requires_grad_(True)
    loss = ml(g, yt)
    loss.backward()
    d["mel24.loss"] = _np(loss)
    d["mel24.grad"] = _np(g.grad)
    # default (fs 22050, 3 res, log10) multi-resolution variant
    mld = mel_mod.MultiMelSpectrogramLoss()
    g = yh.clone().requires_grad_(True)
    loss = mld(g, yt)
    loss.backward()
    d["meldef.loss"] = _np(loss)
    d["meldef.grad"] = _np(g.grad)
    np.savez_compressed(os.path.join(out, "mel.npz"), **d)

    # ---------------- conv layers (layers/conv_layer.py) ----------------
    d = {}
    conv_cases = [
        # name, Cin, Cout, k, stride, dilation, bias, T
        ("first", 1, 8, 7, 1, 1, False, 300),
        ("ru_d1", 8, 8, 7, 1, 1, False, 200),
        ("ru_d3", 8, 8, 7, 1, 3, False, 200),
        ("ru_d9", 16, 16, 7, 1, 9, False, 150),
        ("down3", 8, 16, 6, 3, 1, True, 240),
        ("down5", 16, 24, 10, 5, 1, True, 200),
        ("proj", 32, 16, 3, 1, 1, False, 20),
        ("last", 8, 1, 7, 1, 1, False, 300),
    ]
    for name, ci, co, k, s, dl, b, t in conv_cases:
        m = conv_mod.CausalConv1d(ci, co, k, stride=s, dilation=dl, bias=b)
        xin = torch.randn(2, ci, t, requires_grad=True)
        yo = m(xin)
        gy = torch.randn_like(yo)
        yo.backward(gy)
        d[f"{name}.cfg"] = np.array([ci, co, k, s, dl, int(b), t])
        d[f"{name}.x"] = _np(xin)
        d[f"{name}.w"] = _np(m.conv.weight)
        if b:
            d[f"{name}.b"] = _np(m.conv.bias)
            d[f"{name}.gb"] = _np(m.conv.bias.grad)
        d[f"{name}.y"] = _np(yo)
        d[f"{name}.gy"] = _np(gy)
        d[f"{name}.gx"] = _np(xin.grad)
        d[f"{name}.gw"] = _np(m.conv.weight.grad)
    deconv_cases = [
        ("up5", 16, 8, 5, True, 20),
        ("up3", 8, 4, 3, True, 30),
        ("up4", 12, 8, 4, True, 1),
    ]
    for name, ci, co, s, b, t in deconv_cases:
        m = conv_mod.CausalConvTranspose1d(ci, co, 2 * s, s, bias=b)
        xin = torch.randn(2, ci, t, requires_grad=True)
        yo = m(xin)
        gy = torch.randn_like(yo)
        yo.backward(gy)
        d[f"{name}.cfg"] = np.array([ci, co, 2 * s, s, int(b), t])
        d[f"{name}.x"] = _np(xin)
        d[f"{name}.w"] = _np(m.deconv.weight)
        d[f"{name}.b"] = _np(m.deconv.bias)
        d[f"{name}.y"] = _np(yo)
        d[f"{name}.gy"] = _np(gy)
        d[f"{name}.gx"] = _np(xin.grad)
        d[f"{name}.gw"] = _np(m.deconv.weight.grad)
        d[f"{name}.gb"] = _np(m.deconv.bias.grad)
    # residual unit (models/autoencoder/modules/residual_unit.py:49-80)
    ru_mod = importlib.import_module("models.autoencoder.modules.residual_unit")
    ru = ru_mod.CausalResidualUnit(8, 8, dilation=3)
    xin = torch.randn(2, 8, 180, requires_grad=True)
    yo = ru(xin)
    gy = torch.randn_like(yo)
    yo.backward(gy)
    d.update({"ru.x": _np(xin), "ru.w1": _np(ru.conv1.conv.weight), "ru.w2": _np(ru.conv2.weight),
              "ru.y": _np(yo), "ru.gy": _np(gy), "ru.gx": _np(xin.grad),
              "ru.gw1": _np(ru.conv1.conv.weight.grad), "ru.gw2": _np(ru.conv2.weight.grad)})
    np.savez_compressed(os.path.join(out, "conv.npz"), **d)

    # ---------------- residual VQ (layers/vq_module.py) ----------------
    rvq = vq_mod.ResidualVQ(num_quantizers=4, dim=64, codebook_size=1024)
    rvq.eval()
    z = torch.randn(2, 80, 64) * 2.0
    zg = z.clone().requires_grad_(True)
    q, losses, ppls = rvq(zg)
    r = torch.randn_like(q)
    ((q * r).sum() + losses.sum()).backward()
    d = {"z": _np(z), "q": _np(q), "losses": _np(losses), "ppls": _np(ppls),
         "r": _np(r), "grad_z": _np(zg.grad)}
    for i, layer in enumerate(rvq.layers):
        d[f"embed.{i}"] = _np(layer.embed)
    with torch.no_grad():
        qi, idx = rvq.forward_index(z)
    d["fi.q"] = _np(qi)
    d["fi.idx"] = _np(idx)
    # per-stage top-2 distance margins (near-tie bookkeeping)
    margins = []
    res_ = z.reshape(-1, 64)
    for layer in rvq.layers:
        dist = (res_.pow(2).sum(1, keepdim=True) - 2 * res_ @ layer.embed + layer.embed.pow(2).sum(0, keepdim=True))
        top2 = torch.topk(-dist, 2, dim=1).values
        margins.append(_np(top2[:, 0] - top2[:, 1]))
        ind = (-dist).max(1)[1]
        qq = layer.embed.t()[ind]
        res_ = res_ - (res_ + (qq - res_))
    d["margins"] = np.stack(margins)
    # training-mode VQ (EMA update) on one stage, for the autoencoder trainer path
    vq = vq_mod.VectorQuantize(dim=64, codebook_size=256)
    vq.train()
    e0 = vq.embed.clone()
    zt = torch.randn(160, 64)
    qt, lt, pt = vq(zt)
    d.update({"ema.embed0": _np(e0), "ema.z": _np(zt), "ema.q": _np(qt), "ema.loss": _np(lt),
              "ema.ppl": _np(pt), "ema.embed1": _np(vq.embed), "ema.cluster_size": _np(vq.cluster_size),
              "ema.embed_avg": _np(vq.embed_avg)})
    np.savez_compressed(os.path.join(out, "vq.npz"), **d)

    # ---------------- generators (reduced width) ----------------
    gp = dict(encode_channels=4, decode_channels=4, code_dim=64, codebook_num=2, codebook_size=64)
    mel = mel_mod.MultiMelSpectrogramLoss(**p24)
    T = 2400
    xn = torch.from_numpy(np.stack([clean[0][:T] + 0.1 * noise[0][:T],
                                    clean[1][:T] + 0.1 * noise[1][:T]]).astype(np.float32)).unsqueeze(1)
    xc = torch.from_numpy(np.stack([clean[0][:T], clean[1][:T]])).unsqueeze(1)
    for tag, mod in (("pqc", pqc_mod), ("nopqc", npqc_mod)):
        torch.manual_seed(93)
        G = mod.Generator(**gp)
        d = {"x_noisy": _np(xn), "x_clean": _np(xc)}
        d.update(_sd(G))
        if tag == "pqc":
            G.quantizer.codebook.eval()
            y, zq, z, vql, ppl = G(xn)
            loss = 45.0 * mel(y, xc) + vql.sum()
            d.update({"y": _np(y), "zq": _np(zq), "z": _np(z), "vqloss": _np(vql), "ppl": _np(ppl)})
        else:
            y = G(xn)
            loss = 45.0 * mel(y, xc)
            d["y"] = _np(y)
        loss.backward()
        d["loss"] = _np(loss)
        d.update(_grads(G))
        np.savez_compressed(os.path.join(out, f"generator_{tag}.npz"), **d)

    # ---------------- train_denoise.py step glue (:138-154, :213-243) ----------------
    torch.manual_seed(93)
    G = npqc_mod.Generator(**gp)
    opt = torch.optim.Adam(G.parameters(), lr=5e-5, weight_decay=1e-6)
    d = {"x_noisy": _np(xn), "x_clean": _np(xc)}
    d.update(_sd(G, "sd0."))
    for step in range(2):
        G.train()
        y = G(xn)
        loss = 45.0 * mel(y, xc)
        opt.zero_grad()
        loss.backward()
        tn = torch.nn.utils.clip_grad_norm_(G.parameters(), 1.0)
        opt.step()
        d[f"loss.{step}"] = _np(loss)
        d[f"gradnorm.{step}"] = _np(tn)
        d.update(_sd(G, f"sd{step + 1}."))
    np.savez_compressed(os.path.join(out, "train_step.npz"), **d)

    # ---------------- streaming (AudioDec.py:106-191, conv_layer.py:144-191) ----------------
    make_stream(pqc_mod, clean, noise, gp, out)
    # ---------------- waveform shape loss (losses/waveform_loss.py:15-74) ----------------
    make_waveform(ref, clean, noise, out)

    # ---------------- add_noise (dataloader/data_utils.py:12-22) ----------------
    cl = torch.from_numpy(np.stack([clean[0][:4800], clean[1][:4800]])).unsqueeze(1)
    nz = torch.from_numpy(np.stack([noise[0][:4800], noise[1][:4800]])).unsqueeze(1)
    d = {"clean": _np(cl), "noise": _np(nz)}
    for snr in (10, 15, 19):
        d[f"mixed.{snr}"] = _np(du.add_noise(cl, nz, torch.tensor([snr])))
    np.savez_compressed(os.path.join(out, "add_noise.npz"), **d)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--out", default=HERE)
    ap.add_argument("--only", default=None, help="regenerate one fixture family (stream, waveform, gan, trainer)")
    a = ap.parse_args()
    make(a.ref, a.out, a.only)
    for f in sorted(os.listdir(a.out)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(a.out, f)))
