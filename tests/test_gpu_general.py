"""GPU parity of the layer forms outside the shipped causal configs (sel.genconv):
NonCausalConv1d / NonCausalConvTranspose1d with any stride, padding, dilation,
groups and output_padding, grouped and odd-stride CausalConv1d,
CausalConvTranspose1d with k != 2s (layers/conv_layer.py:26-191), the noncausal
AudioDec generators (mode='noncausal') and the spectral-normalised period
discriminator (models/vocoder/modules/discriminator.py:99-157).

Anchors: reference-generated fixtures (tests/golden/general_conv.npz,
generator_noncausal_*.npz, spectral_norm.npz; make_goldens.py --only general),
which tests/test_oracle_goldens.py also pins the oracle to.  Bounds, norm-wise:
fp32 <= 1e-5 on layer outputs and gradients (2e-5 on the 41-tap layer's weight
gradient: 400-term tap-group sums); bf16 <= 2e-2 against the same fixtures;
generators as tests/test_gpu_model.py (y 1e-5, gradients 5e-3 for the log-mel
adjoint's conditioning)."""
import numpy as np
import pytest
import torch

from conftest import golden

pytestmark = pytest.mark.gpu


def nclose(a, b, rtol, name=""):
    a, b = (v.detach().float().cpu().numpy().astype(np.float64) if torch.is_tensor(v) else np.asarray(v, np.float64)
            for v in (a, b))
    assert a.shape == b.shape, (name, a.shape, b.shape)
    e = np.linalg.norm(a - b) / (np.linalg.norm(b) + 1e-30)
    assert e <= rtol, (name, e)


def _layers():
    from golden.make_goldens import GENERAL_CAUSAL, GENERAL_CAUSALT, GENERAL_CONV, GENERAL_CONVT
    from layers.conv_layer import CausalConv1d, CausalConvTranspose1d, NonCausalConv1d, NonCausalConvTranspose1d
    out = []
    for name, ci, co, k, s, p, dl, g, b, t in GENERAL_CONV:
        out.append((name, lambda ci=ci, co=co, k=k, s=s, p=p, dl=dl, g=g, b=b: NonCausalConv1d(
            ci, co, k, stride=s, padding=p, dilation=dl, groups=g, bias=b), "conv"))
    for name, ci, co, k, s, p, op, g, b, t in GENERAL_CONVT:
        out.append((name, lambda ci=ci, co=co, k=k, s=s, p=p, op=op, g=g, b=b: NonCausalConvTranspose1d(
            ci, co, k, s, padding=p, output_padding=op, groups=g, bias=b), "deconv"))
    for name, ci, co, k, s, dl, g, b, t in GENERAL_CAUSAL:
        out.append((name, lambda ci=ci, co=co, k=k, s=s, dl=dl, g=g, b=b: CausalConv1d(
            ci, co, k, stride=s, dilation=dl, groups=g, bias=b), "conv"))
    for name, ci, co, k, s, t in GENERAL_CAUSALT:
        out.append((name, lambda ci=ci, co=co, k=k, s=s: CausalConvTranspose1d(ci, co, k, s), "deconv"))
    return out


LAYERS = [n for n, _, _ in _layers()]


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
@pytest.mark.parametrize("name", LAYERS)
def test_general_layer_matches_reference_golden(gpu, name, dtype):
    from sel import convops as CO
    g = golden("general_conv")
    make, attr = next((m, a) for n, m, a in _layers() if n == name)
    m = make()
    conv = getattr(m, attr)
    with torch.no_grad():
        conv.weight.copy_(torch.from_numpy(g[f"{name}.w"]))
        if conv.bias is not None:
            conv.bias.copy_(torch.from_numpy(g[f"{name}.b"]))
    m = m.to(gpu)
    x = torch.from_numpy(g[f"{name}.x"]).to(gpu).requires_grad_(True)
    prec = torch.float32 if dtype == "fp32" else torch.bfloat16
    tol = 1e-5 if dtype == "fp32" else 2e-2
    with CO.precision(prec):
        y = m(x)
        nclose(y, g[f"{name}.y"], tol, f"{name}.y")
        y.float().backward(torch.from_numpy(g[f"{name}.gy"]).to(gpu))
    nclose(x.grad, g[f"{name}.gx"], tol, f"{name}.gx")
    nclose(conv.weight.grad, g[f"{name}.gw"], 2 * tol if conv.weight.shape[-1] > 8 else tol, f"{name}.gw")
    if conv.bias is not None:
        nclose(conv.bias.grad, g[f"{name}.gb"], tol, f"{name}.gb")


def test_general_layers_run_native_kernels(gpu):
    """The general forms are HIP launches: the conv primitive's forward, adjoint
    and weight-gradient entry points are called (no torch conv anywhere)."""
    from sel import _lib as L
    from layers.conv_layer import NonCausalConv1d, NonCausalConvTranspose1d
    calls = []
    orig = L.call

    def spy(name, *a, **k):
        calls.append(name)
        return orig(name, *a, **k)
    L.call = spy
    try:
        for m in (NonCausalConv1d(8, 12, 41, stride=4, padding=20, groups=4),
                  NonCausalConvTranspose1d(12, 8, 10, 5)):
            m = m.to(gpu)
            x = torch.randn(2, m.conv.in_channels if hasattr(m, "conv") else 12, 64, device=gpu, requires_grad=True)
            m(x).sum().backward()
    finally:
        L.call = orig
    for entry in ("sel_conv_fwd", "sel_conv_wgrad"):
        assert entry in calls, (entry, sorted(set(calls)))


@pytest.mark.parametrize("tag", ["pqc", "nopqc"])
def test_noncausal_generator_matches_reference_golden(gpu, tag):
    from losses import MultiMelSpectrogramLoss
    if tag == "pqc":
        from models.autoencoder.AudioDec import Generator
    else:
        from models.autoencoder_without_PQC.AudioDec import Generator
    g = golden(f"generator_noncausal_{tag}")
    G = Generator(mode="noncausal", encode_channels=4, decode_channels=4, code_dim=64, codebook_num=2,
                  codebook_size=64)
    sd = {k[3:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("sd.")}
    assert set(sd) == set(G.state_dict()), set(sd) ^ set(G.state_dict())
    G.load_state_dict(sd)
    G = G.to(gpu)
    mel = MultiMelSpectrogramLoss(fs=24000, fft_sizes=[2048], hop_sizes=[300], win_lengths=[None],
                                  num_mels=80, fmin=0, fmax=24000, log_base=None).to(gpu)
    xn = torch.from_numpy(g["x_noisy"]).to(gpu)
    xc = torch.from_numpy(g["x_clean"]).to(gpu)
    if tag == "pqc":
        G.quantizer.codebook.eval()
        y, zq, z, vql, ppl = G(xn)
        nclose(z, g["z"], 1e-5, "z")
        nclose(zq, g["zq"], 1e-5, "zq")
        nclose(vql, g["vqloss"], 1e-4, "vqloss")
        loss = 45.0 * mel(y, xc) + vql.sum()
    else:
        y = G(xn)
        loss = 45.0 * mel(y, xc)
    nclose(y, g["y"], 1e-5, "y")
    nclose(loss, g["loss"], 1e-4, "loss")
    loss.backward()
    n = 0
    for name, p in G.named_parameters():
        key = "g." + name
        if key in g:
            nclose(p.grad, g[key], 5e-3, name)
            n += 1
    assert n > 20


def test_spectral_norm_period_discriminator_matches_reference_golden(gpu):
    from models.vocoder.modules.discriminator import HiFiGANPeriodDiscriminator
    g = golden("spectral_norm")
    D = HiFiGANPeriodDiscriminator(period=3, channels=4, max_downsample_channels=32, use_weight_norm=False,
                                   use_spectral_norm=True)
    sd0 = {k[4:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("sd0.")}
    assert set(sd0) == set(D.state_dict()), set(sd0) ^ set(D.state_dict())
    D.load_state_dict(sd0)
    D = D.to(gpu).train()
    x = torch.from_numpy(g["x"]).to(gpu).requires_grad_(True)
    outs = D(x)
    for j, o in enumerate(outs):
        nclose(o, g[f"out.{j}"], 1e-5, f"out.{j}")
    cot = [torch.randn(o.shape, generator=torch.Generator().manual_seed(j)).to(gpu) for j, o in enumerate(outs)]
    sum((o * c).sum() for o, c in zip(outs, cot)).backward()
    nclose(x.grad, g["grad_x"], 1e-5, "grad_x")
    n = 0
    for name, p in D.named_parameters():
        if "g." + name in g:
            nclose(p.grad, g["g." + name], 1e-5, name)
            n += 1
    assert n == 12   # weight_orig + bias of the 6 convs
    for k, v in D.state_dict().items():
        if k.endswith(("weight_u", "weight_v")):
            nclose(v, g["sd1." + k], 1e-5, k)   # one power iteration per call, as the module pre-hook


def test_grouped_causal_conv_streaming_vs_oracle(gpu):
    """CausalConv1d.inference (conv_layer.py:144-147) for grouped and k != 2s
    strided layers, and CausalConvTranspose1d.inference with k != 2s (:185-188):
    chunk by chunk against the oracle's stream_* restatement."""
    from layers.conv_layer import CausalConv1d, CausalConvTranspose1d
    from oracle import ref_ops as R
    torch.manual_seed(3)
    cases = [(CausalConv1d(8, 8, 7, dilation=2, groups=2), "conv", dict(dilation=2, groups=2)),
             (CausalConv1d(6, 8, 4, stride=3), "conv", dict(stride=3)),
             (CausalConvTranspose1d(6, 6, 7, 3), "deconv", dict(stride=3))]
    for m, kind, kw in cases:
        conv = getattr(m, kind)
        w = conv.weight.detach().clone()
        b = conv.bias.detach().clone() if conv.bias is not None else None
        m = m.to(gpu).eval()
        S = {}
        x = torch.randn(2, conv.in_channels, 60 * 4)
        for c in range(4):
            xc = x[:, :, 60 * c:60 * (c + 1)]
            y = m.inference(xc.to(gpu))
            if kind == "conv":
                yr = R.stream_causal_conv1d(S, "k", xc, w, b, **kw)
            else:
                yr = R.stream_conv_transpose1d(S, "k", xc, w, b, **kw)
            nclose(y, yr, 1e-5, f"{kind}{kw}.{c}")


def test_conv1d_bn_projector_generator_matches_reference_golden(gpu):
    """Generator(projector='conv1d_bn'): the projector's BatchNorm1d on the HIP
    kernels (sel_batchnorm_fwd / _bwd) in training mode — outputs, gradients,
    running statistics, num_batches_tracked — then in evaluation."""
    from losses import MultiMelSpectrogramLoss
    from models.autoencoder.AudioDec import Generator
    g = golden("generator_bn")
    G = Generator(projector="conv1d_bn", encode_channels=4, decode_channels=4, code_dim=64, codebook_num=2,
                  codebook_size=64)
    sd = {k[3:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("sd.")}
    assert set(sd) == set(G.state_dict()), set(sd) ^ set(G.state_dict())
    G.load_state_dict(sd)
    G = G.to(gpu)
    G.quantizer.codebook.eval()
    mel = MultiMelSpectrogramLoss(fs=24000, fft_sizes=[2048], hop_sizes=[300], win_lengths=[None],
                                  num_mels=80, fmin=0, fmax=24000, log_base=None).to(gpu)
    xn = torch.from_numpy(g["x_noisy"]).to(gpu)
    xc = torch.from_numpy(g["x_clean"]).to(gpu)
    y, zq, z, vql, ppl = G(xn)
    nclose(z, g["z"], 1e-5, "z")
    nclose(y, g["y"], 1e-5, "y")
    loss = 45.0 * mel(y, xc) + vql.sum()
    nclose(loss, g["loss"], 1e-4, "loss")
    loss.backward()
    for name, p in G.named_parameters():
        if "g." + name in g:
            nclose(p.grad, g["g." + name], 5e-3, name)
    for k, v in G.state_dict().items():
        if "project.1." in k:
            nclose(v, g["sd1." + k], 1e-6, k)
    G.eval()
    with torch.no_grad():
        y, zq, z, vql, ppl = G(xn)
    nclose(z, g["eval.z"], 1e-5, "eval.z")
    nclose(y, g["eval.y"], 1e-5, "eval.y")


@pytest.mark.parametrize("shape", [(4, 64, 80), (3, 5, 1), (2, 130, 333)])
def test_batchnorm_vs_torch(gpu, shape):
    """sel BatchNorm1d against torch.nn.BatchNorm1d (fp32, the module the
    reference uses) in both modes, with ragged channel counts and T = 1."""
    from sel.bnops import BatchNorm1d
    B, C, T = shape
    torch.manual_seed(5)
    ref = torch.nn.BatchNorm1d(C).to(gpu)
    with torch.no_grad():
        ref.weight.uniform_(0.5, 1.5)
        ref.bias.uniform_(-0.5, 0.5)
    m = BatchNorm1d(C).to(gpu)
    m.load_state_dict(ref.state_dict())
    for step in range(2):
        x = (3.0 * torch.randn(B, C, T, device=gpu) + 1.0)
        xa, xb = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
        ya, yb = m(xa), ref(xb)
        nclose(ya, yb, 1e-5, f"y{step}")
        r = torch.randn_like(yb)
        (ya * r).sum().backward()
        (yb * r).sum().backward()
        nclose(xa.grad, xb.grad, 1e-5, f"gx{step}")
        nclose(m.weight.grad, ref.weight.grad, 1e-5, "gw")
        nclose(m.bias.grad, ref.bias.grad, 1e-5, "gb")
        m.zero_grad()
        ref.zero_grad()
    for k, v in ref.state_dict().items():
        nclose(m.state_dict()[k], v, 1e-6, k)
    m.eval()
    ref.eval()
    x = torch.randn(B, C, T, device=gpu, requires_grad=True)
    x2 = x.detach().clone().requires_grad_(True)
    ya, yb = m(x), ref(x2)
    nclose(ya, yb, 1e-6, "eval.y")
    ya.sum().backward()
    yb.sum().backward()
    nclose(x.grad, x2.grad, 1e-6, "eval.gx")


def _full_noncausal(dev, B=2, T=2400, seed=93):
    from models.autoencoder_without_PQC.AudioDec import Generator
    from oracle import ref_ops as R
    torch.manual_seed(seed)
    G = Generator(mode="noncausal")
    P = {k: v.clone() for k, v in G.state_dict().items()}
    for k, v in P.items():
        if k.endswith("weight") or k.endswith("bias"):
            v.requires_grad_(True)
    x = 0.1 * torch.randn(B, 1, T)
    y = R.generator_forward(P, x, R.generator_geometry(), pqc=False, mode="noncausal")
    r = torch.randn_like(y)
    (y * r).sum().backward()
    return G.to(dev), x, r, y, P


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_full_width_noncausal_generator_vs_oracle(gpu, dtype):
    """The full-width noncausal generator (32 -> 512 channels: the residual units
    on the unfused primitive with the symmetric pad, the k = 2s stride-s
    noncausal down convs and transposed up convs through sel.genconv) against
    the fp32 oracle; bounds as tests/test_gpu_model.py's causal full-width tests."""
    from sel import convops as CO
    G, x, r, y_ref, P = _full_noncausal(gpu)
    prec = torch.float32 if dtype == "fp32" else torch.bfloat16
    ty, tg = (1e-4, 1e-3) if dtype == "fp32" else (5e-2, 1e-1)
    with CO.precision(prec):
        y = G(x.to(gpu))
        nclose(y, y_ref, ty, "y")
        (y.float() * r.to(gpu)).sum().backward()
    n = 0
    for name, p in G.named_parameters():
        if P[name].grad is not None:
            nclose(p.grad, P[name].grad, tg, name)
            n += 1
    assert n > 50


def _cases():
    from test_genconv_host import CONV, CONVT
    return [("conv",) + c for c in CONV] + [("convt",) + c for c in CONVT]


@pytest.mark.parametrize("case", _cases(), ids=lambda c: "_".join(map(str, c)))
def test_genconv_forms_on_the_kernels(gpu, case):
    """sel.genconv through the HIP kernels (fp32) at the host test's shapes,
    edge cases included (one input sample, a 512-row halo, 1-tap strided and
    transposed forms), against torch's fp64 conv / transposed conv on the same
    operands: outputs and all three gradients <= 1e-5 norm-wise."""
    import torch.nn.functional as F
    from sel import genconv as GC
    kind, ci, co, k, s, p, a, g, t = case
    torch.manual_seed(11)
    x = torch.randn(2, t, ci, dtype=torch.float64)
    w = torch.randn((co, ci // g, k) if kind == "conv" else (ci, co // g, k), dtype=torch.float64)
    b = torch.randn(co, dtype=torch.float64)
    xs, ws, bs = (v.clone().requires_grad_(True) for v in (x, w, b))
    if kind == "conv":
        ref = F.conv1d(xs.transpose(1, 2), ws, bs, s, p, a, g).transpose(1, 2)
    else:
        ref = F.conv_transpose1d(xs.transpose(1, 2), ws, bs, s, p, a, g).transpose(1, 2)
    r = torch.randn_like(ref)
    (ref * r).sum().backward()
    xg, wg, bg = (v.float().to(gpu).requires_grad_(True) for v in (x, w, b))
    if kind == "conv":
        y = GC.conv1d(xg.contiguous(), wg, bg, s, p, a, g)
    else:
        y = GC.conv_transpose1d(xg.contiguous(), wg, bg, s, p, a, g)
    nclose(y, ref, 1e-5, "y")
    (y * r.float().to(gpu)).sum().backward()
    for name, got, want in (("gx", xg.grad, xs.grad), ("gw", wg.grad, ws.grad), ("gb", bg.grad, bs.grad)):
        nclose(got, want, 1e-5, name)
