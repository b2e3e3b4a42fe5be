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
