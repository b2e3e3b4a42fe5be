"""ORACLE / TEST INFRASTRUCTURE — never imported by the product path.

Op-for-op PyTorch-CPU restatement of the reference's denoise-training hot path
(s194584/dl-speech-enhancement).  Only ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg may import this module, and only as the
checker / the timed CPU baseline — never as the thing measured or shipped.

It is pinned against golden vectors produced by importing the reference itself
in the build container (tests/golden/make_goldens.py -> tests/golden/*.npz,
checked by tests/test_oracle_goldens.py).

Everything is functional (plain tensors + a flat parameter dict keyed exactly
like the reference ``state_dict``) so it can run from fixtures without the
reference module tree.  Each function cites the reference lines it restates.
"""
import math

import torch
import torch.nn.functional as F


# --------------------------------------------------------------------------
# spectral losses  (losses/stft_loss.py, losses/mel_loss.py)
# --------------------------------------------------------------------------

def hann(win_length):
    """Periodic Hann window buffer: losses/stft_loss.py:97, mel_loss.py:49."""
    return torch.hann_window(win_length)


def stft_mag(x, fft_size, hop_size, win_length, window, eps=1e-7):
    """losses/stft_loss.py:19-35 — |STFT| with power floor, (B, frames, bins)."""
    z = torch.stft(x, fft_size, hop_size, win_length, window, return_complex=True)
    p = z.real ** 2 + z.imag ** 2
    return torch.sqrt(torch.clamp(p, min=eps)).transpose(2, 1)


def htk_melscale_fbanks(n_freqs, f_min, f_max, n_mels, sample_rate):
    """torchaudio 2.1.1 functional.melscale_fbanks(norm=None, mel_scale="htk")
    (third-party, absent here: restated from its published algorithm; parity of
    mel_spectrogram.py:38 is therefore unpinned beyond this restatement).
    fp32 throughout, as torchaudio: linspace freqs, HTK mel points, triangles."""
    all_freqs = torch.linspace(0, sample_rate // 2, n_freqs)
    m_min = 2595.0 * math.log10(1.0 + (f_min / 700.0))
    m_max = 2595.0 * math.log10(1.0 + (f_max / 700.0))
    m_pts = torch.linspace(m_min, m_max, n_mels + 2)
    f_pts = 700.0 * (10.0 ** (m_pts / 2595.0) - 1.0)
    f_diff = f_pts[1:] - f_pts[:-1]
    slopes = f_pts.unsqueeze(0) - all_freqs.unsqueeze(1)
    down = (-1.0 * slopes[:, :-2]) / f_diff[:-1]
    up = slopes[:, 2:] / f_diff[1:]
    return torch.max(torch.zeros(1), torch.min(down, up))  # (n_freqs, n_mels)


def power_melspec(x, sample_rate=48000, n_fft=400, hop_length=None, win_length=None, n_mels=128, f_min=0.0,
                  f_max=None, power=2.0):
    """mel_spectrogram.py:38 — torchaudio transforms.MelSpectrogram(48000) with its
    defaults: Spectrogram(center, reflect, periodic Hann, onesided, |X|^power)
    then MelScale (HTK, no norm).  x (..., T) -> (..., n_mels, 1 + T // hop)."""
    win_length = win_length or n_fft
    hop_length = hop_length or win_length // 2
    f_max = f_max if f_max is not None else float(sample_rate // 2)
    shape = x.shape
    x2 = x.reshape(-1, shape[-1])
    z = torch.stft(x2, n_fft, hop_length, win_length, torch.hann_window(win_length), center=True,
                   pad_mode="reflect", normalized=False, onesided=True, return_complex=True)
    spec = z.abs().pow(power)  # (N, K, F)
    fb = htk_melscale_fbanks(n_fft // 2 + 1, f_min, f_max, n_mels, sample_rate)
    mel = torch.matmul(spec.transpose(-1, -2), fb).transpose(-1, -2)
    return mel.reshape(shape[:-1] + mel.shape[-2:])


def mel_l1(pred, target, **kw):
    """mel_spectrogram.py:40-44 Mel_L1: nn.L1Loss()(mel(pred), mel(target))."""
    return F.l1_loss(power_melspec(pred, **kw), power_melspec(target, **kw))


def spectral_convergence(x_mag, y_mag):
    """losses/stft_loss.py:45-56 — global Frobenius ratio."""
    return torch.norm(y_mag - x_mag, p="fro") / torch.norm(y_mag, p="fro")


def log_stft_magnitude(x_mag, y_mag):
    """losses/stft_loss.py:66-77 — mean |ln y - ln x|."""
    return F.l1_loss(torch.log(y_mag), torch.log(x_mag))


def stft_loss(x, y, fft_size, hop_size, win_length, window):
    """losses/stft_loss.py:100-117 -> (sc, mag)."""
    xm = stft_mag(x, fft_size, hop_size, win_length, window)
    ym = stft_mag(y, fft_size, hop_size, win_length, window)
    return spectral_convergence(xm, ym), log_stft_magnitude(xm, ym)


def mr_stft_loss(x, y, resolutions, windows):
    """losses/stft_loss.py:146-170 — mean over resolutions of (sc, mag)."""
    if x.dim() == 3:
        x = x.reshape(-1, x.size(2))
        y = y.reshape(-1, y.size(2))
    sc_total, mag_total = 0.0, 0.0
    for (n, h, w), win in zip(resolutions, windows):
        sc, mg = stft_loss(x, y, n, h, w, win)
        sc_total = sc_total + sc
        mag_total = mag_total + mg
    return sc_total / len(resolutions), mag_total / len(resolutions)


def _log_fn(log_base):
    if log_base is None:
        return torch.log
    if log_base == 2.0:
        return torch.log2
    if log_base == 10.0:
        return torch.log10
    raise ValueError(log_base)


def melspec(x, fft_size, hop_size, win_length, window, melmat, eps=1e-10, log_base=10.0):
    """losses/mel_loss.py:74-94 — log-mel (B, mels, frames)."""
    if x.dim() == 3:
        x = x.reshape(-1, x.size(2))
    z = torch.stft(x, fft_size, hop_size, win_length, window, return_complex=True)
    p = z.real ** 2 + z.imag ** 2
    amp = torch.sqrt(torch.clamp(p, min=eps)).transpose(2, 1)
    m = torch.clamp(torch.matmul(amp, melmat), min=eps)
    return _log_fn(log_base)(m).transpose(1, 2)


def multi_mel_loss(y_hat, y, resolutions, windows, melmats, eps=1e-10, log_base=10.0):
    """losses/mel_loss.py:140-155 — mean over resolutions of L1(mel(y_hat), mel(y))."""
    total = 0.0
    for (n, h, w), win, mm in zip(resolutions, windows, melmats):
        total = total + F.l1_loss(melspec(y_hat, n, h, w, win, mm, eps, log_base),
                                  melspec(y, n, h, w, win, mm, eps, log_base))
    return total / len(resolutions)


# --------------------------------------------------------------------------
# conv layers  (layers/conv_layer.py)
# --------------------------------------------------------------------------

def causal_conv1d(x, w, b=None, stride=1, dilation=1):
    """layers/conv_layer.py:139-142 — left zero pad (k-1)*d then valid conv."""
    k = w.shape[-1]
    x = F.pad(x, ((k - 1) * dilation, 0))
    return F.conv1d(x, w, b, stride=stride, dilation=dilation)


def causal_conv_transpose1d(x, w, b=None, stride=1):
    """layers/conv_layer.py:180-183 — replicate-pad 1 left, deconv, crop [s:-s]."""
    x = torch.cat([x[:, :, :1], x], dim=-1)
    y = F.conv_transpose1d(x, w, b, stride=stride)
    return y[:, :, stride:-stride]


def noncausal_conv1d(x, w, b=None, stride=1, padding=-1, dilation=1, groups=1):
    """layers/conv_layer.py:26-65 — nn.Conv1d with padding (k-1)//2*d by default."""
    if padding < 0:
        padding = (w.shape[-1] - 1) // 2 * dilation
    return F.conv1d(x, w, b, stride=stride, padding=padding, dilation=dilation, groups=groups)


def noncausal_conv_transpose1d(x, w, b=None, stride=1, padding=-1, output_padding=-1, groups=1):
    """layers/conv_layer.py:68-106 — nn.ConvTranspose1d, padding (s+1)//2 and
    output_padding s % 2 by default."""
    if padding < 0:
        padding = (stride + 1) // 2
    if output_padding < 0:
        output_padding = 1 if stride % 2 else 0
    return F.conv_transpose1d(x, w, b, stride=stride, padding=padding, output_padding=output_padding,
                              groups=groups)


def grouped_causal_conv1d(x, w, b=None, stride=1, dilation=1, groups=1):
    """layers/conv_layer.py:109-142 with groups: left zero pad (k-1)*d, conv."""
    k = w.shape[-1]
    return F.conv1d(F.pad(x, ((k - 1) * dilation, 0)), w, b, stride=stride, dilation=dilation, groups=groups)


def elu(x):
    """nn.ELU(alpha=1): models/autoencoder/modules/residual_unit.py:32."""
    return F.elu(x)


def residual_unit(x, w1, w2, dilation, mode="causal"):
    """residual_unit.py:43-46 — x + conv1x1(ELU(conv_k7_d(ELU(x)))), conv1
    causal (:49-76) or noncausal with 'same' padding (:20-41)."""
    if mode == "causal":
        y = causal_conv1d(elu(x), w1, None, 1, dilation)
    else:
        y = noncausal_conv1d(elu(x), w1, None, 1, -1, dilation)
    y = F.conv1d(elu(y), w2)
    return x + y


# --------------------------------------------------------------------------
# residual VQ  (layers/vq_module.py)
# --------------------------------------------------------------------------

def vq_distance(flatten, embed):
    """vq_module.py:64-68 — evaluation order as written in the reference."""
    return (flatten.pow(2).sum(1, keepdim=True)
            - 2 * flatten @ embed
            + embed.pow(2).sum(0, keepdim=True))


def vq_forward(inp, embed, commitment=1.0):
    """vq_module.py:61-88 in eval mode (no EMA: trainer/denoise.py:60).

    Returns (quantize_st, loss, perplexity, indices)."""
    dim = embed.shape[0]
    n_embed = embed.shape[1]
    flatten = inp.reshape(-1, dim)
    dist = vq_distance(flatten, embed)
    _, ind = (-dist).max(1)
    onehot = F.one_hot(ind, n_embed).type(inp.dtype)
    ind = ind.view(*inp.shape[:-1])
    q = F.embedding(ind, embed.transpose(0, 1))
    loss = F.mse_loss(q.detach(), inp) * commitment
    q = inp + (q - inp).detach()
    p = onehot.mean(0)
    ppl = torch.exp(-torch.sum(p * torch.log(p + 1e-10)))
    return q, loss, ppl, ind


def rvq_forward(x, embeds):
    """vq_module.py:119-134 — residual not detached (:129)."""
    out = 0.0
    residual = x
    losses, ppls, inds = [], [], []
    for e in embeds:
        q, l, p, i = vq_forward(residual, e)
        residual = residual - q
        out = out + q
        losses.append(l)
        ppls.append(p)
        inds.append(i)
    return out, torch.stack(losses), torch.stack(ppls), torch.stack(inds)


# --------------------------------------------------------------------------
# AudioDec generator (models/autoencoder*/)
# --------------------------------------------------------------------------

def generator_geometry(encode_channels=32, decode_channels=32, enc_ratios=(2, 4, 8, 16),
                       dec_ratios=(16, 8, 4, 2), enc_strides=(3, 4, 5, 5),
                       dec_strides=(5, 5, 4, 3), **_):
    """Channel/stride plan of encoder.py:84-110 and decoder.py:84-114."""
    enc = []
    cin = encode_channels
    for r, s in zip(enc_ratios, enc_strides):
        enc.append((cin, encode_channels * r, s))
        cin = encode_channels * r
    dec = []
    for i, s in enumerate(dec_strides):
        ci = decode_channels * dec_ratios[i]
        co = decode_channels * dec_ratios[i + 1] if i < len(dec_ratios) - 1 else decode_channels
        dec.append((ci, co, s))
    return enc, dec


def _conv(mode):
    """The mode's Conv1d (encoder.py:38-45, decoder.py:38-45, projector.py:31-37)."""
    if mode == "causal":
        return causal_conv1d
    return lambda x, w, b=None, stride=1, dilation=1: noncausal_conv1d(x, w, b, stride, -1, dilation)


def encoder_forward(P, x, geo, dilations=(1, 3, 9), mode="causal"):
    """encoder.py:112-116 / EncoderBlock :61-65 (mode 'causal' or 'noncausal')."""
    enc, _ = geo
    conv = _conv(mode)
    h = conv(x, P["encoder.conv.conv.weight"])
    for i, (ci, co, s) in enumerate(enc):
        pre = f"encoder.conv_blocks.{i}"
        for j, d in enumerate(dilations):
            ru = f"{pre}.res_units.{j}"
            h = residual_unit(h, P[f"{ru}.conv1.conv.weight"], P[f"{ru}.conv2.weight"], d, mode)
        h = conv(h, P[f"{pre}.conv.conv.weight"], P.get(f"{pre}.conv.conv.bias"), stride=s)
    return h


def decoder_forward(P, z, geo, pqc=True, dilations=(1, 3, 9), mode="causal"):
    """decoder.py:116-121 (PQC) / without_PQC decoder.py:116-123 (conv1 skipped)."""
    _, dec = geo
    conv = _conv(mode)
    convt = causal_conv_transpose1d if mode == "causal" else noncausal_conv_transpose1d
    h = conv(z, P["decoder.conv1.conv.weight"]) if pqc else z
    for i, (ci, co, s) in enumerate(dec):
        pre = f"decoder.conv_blocks.{i}"
        h = convt(h, P[f"{pre}.conv.deconv.weight"], P.get(f"{pre}.conv.deconv.bias"), s)
        for j, d in enumerate(dilations):
            ru = f"{pre}.res_units.{j}"
            h = residual_unit(h, P[f"{ru}.conv1.conv.weight"], P[f"{ru}.conv2.weight"], d, mode)
    return conv(h, P["decoder.conv2.conv.weight"])


def batch_norm1d(x, w, b, running_mean, running_var, training=True, momentum=0.1, eps=1e-5):
    """torch.nn.BatchNorm1d on (B, C, T) (projector.py:40-44, model='conv1d_bn'),
    restated: training normalises with the batch mean and biased variance and
    returns the momentum-updated running statistics (unbiased variance);
    evaluation uses the running statistics.  Returns (y, running_mean', running_var')."""
    if training:
        n = x.shape[0] * x.shape[2]
        mean = x.mean((0, 2))
        var = ((x - mean.view(1, -1, 1)) ** 2).mean((0, 2))
        with torch.no_grad():
            rm = (1 - momentum) * running_mean + momentum * mean
            rv = (1 - momentum) * running_var + momentum * var * n / (n - 1)
    else:
        mean, var, rm, rv = running_mean, running_var, running_mean, running_var
    y = (x - mean.view(1, -1, 1)) / torch.sqrt(var.view(1, -1, 1) + eps)
    return y * w.view(1, -1, 1) + b.view(1, -1, 1), rm, rv


def generator_forward(P, x, geo, pqc=True, codebook_num=8, mode="causal", training=True):
    """AudioDec.py:95-103 (PQC) or autoencoder_without_PQC/AudioDec.py:94-100.
    A 'conv1d_bn' projector (projector.project.1.* keys) runs its BatchNorm1d in
    `training` mode; the updated running statistics are written back into P."""
    h = encoder_forward(P, x, geo, mode=mode)
    if not pqc:
        return decoder_forward(P, h, geo, pqc=False, mode=mode)
    if "projector.project.1.weight" in P:
        z = _conv(mode)(h, P["projector.project.0.conv.weight"])
        pre = "projector.project.1"
        z, P[pre + ".running_mean"], P[pre + ".running_var"] = batch_norm1d(
            z, P[pre + ".weight"], P[pre + ".bias"], P[pre + ".running_mean"], P[pre + ".running_var"], training)
    else:
        z = _conv(mode)(h, P["projector.project.conv.weight"])
    embeds = [P[f"quantizer.codebook.layers.{i}.embed"] for i in range(codebook_num)]
    zq, vql, ppl, _ = rvq_forward(z.transpose(2, 1), embeds)
    zq = zq.transpose(2, 1)
    y = decoder_forward(P, zq, geo, pqc=True, mode=mode)
    return y, zq, z, vql, ppl


# --------------------------------------------------------------------------
# streaming  (layers/conv_layer.py:144-191, models/autoencoder/AudioDec.py:106-191)
# --------------------------------------------------------------------------

def stream_causal_conv1d(S, key, x, w, b=None, stride=1, dilation=1, groups=1):
    """conv_layer.py:144-147 — conv over cat(pad_buffer, x); keep the last (k-1)d."""
    pad = (w.shape[-1] - 1) * dilation
    buf = S.get(key, torch.zeros(x.shape[0], x.shape[1], pad, dtype=x.dtype))
    xb = torch.cat([buf, x], -1)
    S[key] = xb[:, :, -pad:]
    return F.conv1d(xb, w, b, stride=stride, dilation=dilation, groups=groups)


def stream_conv_transpose1d(S, key, x, w, b=None, stride=1):
    """conv_layer.py:185-188 — deconv(cat(pad_buffer, x))[s:-s]; keep the last sample."""
    buf = S.get(key, torch.zeros(x.shape[0], x.shape[1], 1, dtype=x.dtype))
    xb = torch.cat([buf, x], -1)
    S[key] = xb[:, :, -1:]
    return F.conv_transpose1d(xb, w, b, stride=stride)[:, :, stride:-stride]


def stream_residual_unit(S, key, x, w1, w2, dilation):
    """residual_unit.py:78-81 — conv1 streams, the 1x1 conv2 does not."""
    y = stream_causal_conv1d(S, key, elu(x), w1, None, 1, dilation)
    return x + F.conv1d(elu(y), w2)


def stream_encode(P, S, x, geo, dilations=(1, 3, 9), project=True):
    """AudioDec.py:160-166 -> encoder.py:118-123, projector.py:52-54 (without_PQC
    AudioDec.py:160-166: encoder only, project=False)."""
    enc, _ = geo
    h = stream_causal_conv1d(S, "encoder.conv", x, P["encoder.conv.conv.weight"])
    for i, (ci, co, s) in enumerate(enc):
        pre = f"encoder.conv_blocks.{i}"
        for j, d in enumerate(dilations):
            ru = f"{pre}.res_units.{j}"
            h = stream_residual_unit(S, f"{ru}.conv1", h, P[f"{ru}.conv1.conv.weight"], P[f"{ru}.conv2.weight"], d)
        h = stream_causal_conv1d(S, f"{pre}.conv", h, P[f"{pre}.conv.conv.weight"], P.get(f"{pre}.conv.conv.bias"),
                                 stride=s)
    if not project:
        return h
    return stream_causal_conv1d(S, "projector.project", h, P["projector.project.conv.weight"])


def stream_quantize(z, embeds):
    """quantizer.py:42-44 -> vq_module.py:136-149 with flatten_idx: stage i's index + K*i."""
    _, _, _, inds = rvq_forward(z.transpose(2, 1), embeds)
    K = embeds[0].shape[1]
    inds = inds + K * torch.arange(len(embeds)).view(-1, *([1] * (inds.dim() - 1)))
    return inds.squeeze(1)


def stream_lookup(idx, embeds):
    """vq_module.py:151-162: sum over stages of the flattened codebook rows."""
    book = torch.cat([e.transpose(0, 1) for e in embeds], 0)
    return F.embedding(idx, book).sum(0, keepdim=True)


def stream_decode(P, S, zq, geo, dilations=(1, 3, 9), pqc=True):
    """AudioDec.py:178-179 -> decoder.py:123-128 on zq (B, L, D); without_PQC
    decoder.py:125-132 skips conv1."""
    _, dec = geo
    h = zq.transpose(2, 1)
    if pqc:
        h = stream_causal_conv1d(S, "decoder.conv1", h, P["decoder.conv1.conv.weight"])
    for i, (ci, co, s) in enumerate(dec):
        pre = f"decoder.conv_blocks.{i}"
        h = stream_conv_transpose1d(S, f"{pre}.conv", h, P[f"{pre}.conv.deconv.weight"],
                                    P.get(f"{pre}.conv.deconv.bias"), s)
        for j, d in enumerate(dilations):
            ru = f"{pre}.res_units.{j}"
            h = stream_residual_unit(S, f"{ru}.conv1", h, P[f"{ru}.conv1.conv.weight"], P[f"{ru}.conv2.weight"], d)
    return stream_causal_conv1d(S, "decoder.conv2", h, P["decoder.conv2.conv.weight"])


# --------------------------------------------------------------------------
# waveform shape loss  (losses/waveform_loss.py:15-74)
# --------------------------------------------------------------------------

def waveform_shape_loss(y_hat, y, winlen):
    """waveform_loss.py:26-38 — L1(maxpool_w(|y_hat|), maxpool_w(|y|))."""
    return F.l1_loss(F.max_pool1d(torch.abs(y_hat), winlen), F.max_pool1d(torch.abs(y), winlen))


def multi_window_shape_loss(y_hat, y, winlen=(300, 200, 100)):
    """waveform_loss.py:58-74 — mean over the window lengths."""
    loss = 0.0
    for w in winlen:
        loss = loss + waveform_shape_loss(y_hat, y, w)
    return loss / len(winlen)


# --------------------------------------------------------------------------
# data pipeline  (dataloader/AudioDataset.py:25-36 -> torchaudio.functional.resample)
# --------------------------------------------------------------------------

def resample(x, orig_freq, new_freq, lowpass_filter_width=6, rolloff=0.99):
    """torchaudio 2.1.1 functional.resample, sinc_interp_hann (third-party, absent
    here: restated from its published _get_sinc_resample_kernel /
    _apply_sinc_resample_kernel; parity unpinned by any reference fixture)."""
    if orig_freq == new_freq:
        return x
    g = math.gcd(int(orig_freq), int(new_freq))
    o, n = int(orig_freq) // g, int(new_freq) // g
    base = min(o, n) * rolloff
    width = math.ceil(lowpass_filter_width * o / base)
    idx = torch.arange(-width, width + o, dtype=torch.float64)[None, None] / o
    t = torch.arange(0, -n, -1, dtype=torch.float64)[:, None, None] / n + idx
    t = (t * base).clamp(-lowpass_filter_width, lowpass_filter_width)
    window = torch.cos(t * math.pi / lowpass_filter_width / 2) ** 2
    t = t * math.pi
    kern = torch.where(t == 0, torch.ones_like(t), torch.sin(t) / t) * window * (base / o)
    shape = x.shape
    w = x.reshape(-1, shape[-1]).double()
    length = w.shape[-1]
    w = F.pad(w, (width, width + o))
    y = F.conv1d(w[:, None], kern, stride=o).transpose(1, 2).reshape(w.shape[0], -1)
    target = math.ceil(n * length / o)
    return y[..., :target].reshape(*shape[:-1], target).to(x.dtype)


# --------------------------------------------------------------------------
# step glue  (dataloader/data_utils.py, train_denoise.py, trainerGAN.py)
# --------------------------------------------------------------------------

def add_noise(speech, noise, snr):
    """dataloader/data_utils.py:12-22 — batch-global norms, math.exp(snr/10)."""
    assert speech.shape == noise.shape
    sp = speech.norm(p=2)
    npow = noise.norm(p=2)
    scale = math.exp(snr / 10) * npow / sp
    return (scale * speech + noise) / 2


def snr_db(preds, target):
    """torchmetrics 1.2.0 SignalNoiseRatio (zero_mean=False), mean over batch.

    Third-party, absent here: parity unpinned (restated from its published
    formula 10*log10((sum t^2 + eps) / (sum (t-p)^2 + eps)), eps=finfo.eps)."""
    eps = torch.finfo(preds.dtype).eps
    noise = target - preds
    v = (torch.sum(target ** 2, dim=-1) + eps) / (torch.sum(noise ** 2, dim=-1) + eps)
    return (10 * torch.log10(v)).mean()


# --------------------------------------------------------------------------
# HiFi-GAN MSD + MPD discriminator  (models/vocoder/HiFiGAN.py:308-395,
# models/vocoder/modules/discriminator.py:26-447) and the GAN losses
# (losses/adversarial_loss.py:13-124, losses/feat_match_loss.py:13-55)
# --------------------------------------------------------------------------

def spectral_norm_weight(w_orig, u, v, training=True, eps=1e-12):
    """torch.nn.utils.spectral_norm(n_power_iterations=1, dim=0) as applied by
    discriminator.py:150-157, restated: in training one power iteration
    v = normalize(W^T u), u = normalize(W v) on W = w_orig.flatten(1), then
    w = w_orig / (u . W v).  Returns (w, u', v')."""
    W = w_orig.flatten(1)
    if training:
        with torch.no_grad():   # u, v are constants of the backward (torch clones them)
            v = F.normalize(torch.mv(W.t(), u), dim=0, eps=eps)
            u = F.normalize(torch.mv(W, v), dim=0, eps=eps)
    sigma = torch.dot(u, torch.mv(W, v))
    return w_orig / sigma, u, v


def _wn(P, key):
    """torch.nn.utils.weight_norm(dim=0): w = g * v / ||v|| (norm over all dims but 0);
    spectral-norm keys (weight_orig / weight_u / weight_v): one training-mode step."""
    if key + ".weight" in P:
        return P[key + ".weight"]
    if key + ".weight_orig" in P:
        return spectral_norm_weight(P[key + ".weight_orig"], P[key + ".weight_u"], P[key + ".weight_v"])[0]
    g, v = P[key + ".weight_g"], P[key + ".weight_v"]
    return g * v / v.flatten(1).norm(dim=1).view(-1, *([1] * (v.dim() - 1)))


def scale_discriminator_plan(in_channels=1, out_channels=1, kernel_sizes=(15, 41, 5, 3), channels=128,
                             max_downsample_channels=1024, max_groups=16, downsample_scales=(2, 2, 4, 4, 1),
                             **_):
    """Layer plan of HiFiGANScaleDiscriminator.__init__ (discriminator.py:257-324):
    (cin, cout, k, stride, pad, groups, leaky) per layer."""
    plan = [(in_channels, channels, kernel_sizes[0], 1, (kernel_sizes[0] - 1) // 2, 1, True)]
    cin, cout, groups = channels, channels, 4
    for s in downsample_scales:
        plan.append((cin, cout, kernel_sizes[1], s, (kernel_sizes[1] - 1) // 2, groups, True))
        cin = cout
        cout = min(cin * 2, max_downsample_channels)
        groups = min(groups * 4, max_groups)
    cout = min(cin * 2, max_downsample_channels)
    plan.append((cin, cout, kernel_sizes[2], 1, (kernel_sizes[2] - 1) // 2, 1, True))
    plan.append((cout, out_channels, kernel_sizes[3], 1, (kernel_sizes[3] - 1) // 2, 1, False))
    return plan


def period_discriminator_plan(in_channels=1, out_channels=1, kernel_sizes=(5, 3), channels=32,
                              downsample_scales=(3, 3, 3, 3, 1), max_downsample_channels=1024, **_):
    """Layer plan of HiFiGANPeriodDiscriminator.__init__ (discriminator.py:69-97):
    (cin, cout, k, stride, pad, leaky); the output conv uses kernel k1 - 1 with
    padding (k1 - 1) // 2 (:91-97, as written)."""
    plan = []
    cin, cout = in_channels, channels
    for s in downsample_scales:
        plan.append((cin, cout, kernel_sizes[0], s, (kernel_sizes[0] - 1) // 2, True))
        cin = cout
        cout = min(cout * 4, max_downsample_channels)
    plan.append((cout, out_channels, kernel_sizes[1] - 1, 1, (kernel_sizes[1] - 1) // 2, False))
    return plan


def scale_discriminator(P, pre, x, plan, slope=0.1):
    """HiFiGANScaleDiscriminator.forward (:337-352): every layer's output is kept."""
    outs = []
    for i, (ci, co, k, s, p, g, leaky) in enumerate(plan):
        key = f"{pre}.layers.{i}.0" if leaky else f"{pre}.layers.{i}"
        x = F.conv1d(x, _wn(P, key), P.get(key + ".bias"), stride=s, padding=p, groups=g)
        if leaky:
            x = F.leaky_relu(x, slope)
        outs.append(x)
    return outs


def period_discriminator(P, pre, x, period, plan, slope=0.1):
    """HiFiGANPeriodDiscriminator.forward (:110-137): reflect-pad T to a multiple
    of the period, view (B, C, T/p, p), (k, 1) Conv2d stack, flatten the last."""
    b, c, t = x.shape
    if t % period:
        n_pad = period - t % period
        x = F.pad(x, (0, n_pad), "reflect")
        t += n_pad
    x = x.view(b, c, t // period, period)
    outs = []
    n = len(plan)
    for i, (ci, co, k, s, p, leaky) in enumerate(plan):
        key = f"{pre}.convs.{i}.0" if i < n - 1 else f"{pre}.output_conv"
        x = F.conv2d(x, _wn(P, key), P.get(key + ".bias"), stride=(s, 1), padding=(p, 0))
        if leaky:
            x = F.leaky_relu(x, slope)
        outs.append(x)
    outs[-1] = torch.flatten(outs[-1], 1, -1)
    return outs


def hifigan_discriminator(P, x, scales=3, scale_downsample_pooling_params=None, scale_discriminator_params=None,
                          periods=(2, 3, 5, 7, 11), period_discriminator_params=None, **_):
    """HiFiGAN.Discriminator.forward (HiFiGAN.py:380-395): MSD outputs (AvgPool1d
    between scales, discriminator.py:432-447) followed by MPD outputs (:195-209)."""
    pool = scale_downsample_pooling_params or {"kernel_size": 4, "stride": 2, "padding": 2}
    sp = scale_discriminator_params or {}
    pp = period_discriminator_params or {}
    b, c, t = x.shape
    if c != 1:
        x = x.reshape(b * c, 1, t)
    splan = scale_discriminator_plan(**sp)
    slope = sp.get("nonlinear_activation_params", {}).get("negative_slope", 0.1)
    outs = []
    h = x
    for i in range(scales):
        outs.append(scale_discriminator(P, f"msd.discriminators.{i}", h, splan, slope))
        h = F.avg_pool1d(h, **pool)
    pplan = period_discriminator_plan(**pp)
    pslope = pp.get("nonlinear_activation_params", {}).get("negative_slope", 0.1)
    for i, p in enumerate(periods):
        outs.append(period_discriminator(P, f"mpd.discriminators.{i}", x, p, pplan, pslope))
    return outs


def generator_adv_loss(outputs, average_by_discriminators=True, loss_type="mse"):
    """GeneratorAdversarialLoss.forward (adversarial_loss.py:30-58)."""
    crit = (lambda v: F.mse_loss(v, v.new_ones(v.size()))) if loss_type == "mse" else (lambda v: -v.mean())
    if isinstance(outputs, (tuple, list)):
        loss = 0.0
        for i, o in enumerate(outputs):
            if isinstance(o, (tuple, list)):
                o = o[-1]
            loss = loss + crit(o)
        if average_by_discriminators:
            loss = loss / (i + 1)
        return loss
    return crit(outputs)


def discriminator_adv_loss(outputs_hat, outputs, average_by_discriminators=True, loss_type="mse"):
    """DiscriminatorAdversarialLoss.forward (adversarial_loss.py:81-124) -> (real, fake)."""
    if loss_type == "mse":
        real_c = lambda v: F.mse_loss(v, v.new_ones(v.size()))  # noqa: E731
        fake_c = lambda v: F.mse_loss(v, v.new_zeros(v.size()))  # noqa: E731
    else:
        real_c = lambda v: -torch.mean(torch.min(v - 1, v.new_zeros(v.size())))  # noqa: E731
        fake_c = lambda v: -torch.mean(torch.min(-v - 1, v.new_zeros(v.size())))  # noqa: E731
    if isinstance(outputs, (tuple, list)):
        real = fake = 0.0
        for i, (oh, o) in enumerate(zip(outputs_hat, outputs)):
            if isinstance(oh, (tuple, list)):
                oh, o = oh[-1], o[-1]
            real = real + real_c(o)
            fake = fake + fake_c(oh)
        if average_by_discriminators:
            real, fake = real / (i + 1), fake / (i + 1)
        return real, fake
    return real_c(outputs), fake_c(outputs_hat)


def feat_match_loss(feats_hat, feats, average_by_layers=True, average_by_discriminators=True,
                    include_final_outputs=False):
    """FeatureMatchLoss.forward (feat_match_loss.py:29-55)."""
    total = 0.0
    for i, (fh, f) in enumerate(zip(feats_hat, feats)):
        part = 0.0
        if not include_final_outputs:
            fh, f = fh[:-1], f[:-1]
        for j, (a, b) in enumerate(zip(fh, f)):
            part = part + F.l1_loss(a, b.detach())
        if average_by_layers:
            part = part / (j + 1)
        total = total + part
    if average_by_discriminators:
        total = total / (i + 1)
    return total
