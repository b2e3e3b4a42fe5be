"""Every kernel-variant knob that still selects compiled code (include/sel.h
sel_tune; DESIGN.md §6 lists them) against the default path, at the configs'
own layer shapes.  Knobs covered elsewhere: 0 and 47/50/51/52 (tile variants
and the sample-tile kernel, test_gpu_c3), 1/3/4/5/11/54/55 (test_gpu_conv; 54 /
55: the fp32 kernels), 2 and 39 (RVQ kernels, test_gpu_model), 9/18/19/21/22/26/
30 (discriminator variants, test_gpu_dconv_variants / test_gpu_c5), 24
(test_gpu_conv).  The rest are here:

* generator (C3 widths, B = 2 x 1 s @ 24 kHz, bf16, full fwd + bwd): 6 (thin
  kernel instances on their alternative tile rows), 7 (thin kernel off: tiled
  kernels), 8 (plain 2-D grid instead of the XCD-aware order), 12 (epilogue
  prefetch flipped on every thin instance), 20 (two-pass split reduction),
  40 (k_ru64_bwdw workgroup target: another split of the weight-gradient
  rows), 41 (the 64-channel backward without gh on the eight-wave kernel
  instead of k_ru64_bwd: bit-identical), 56 (128-row tiles for k_ru32_fwd),
  57 (the two-set fragment pipeline of k_wgrad3_bf16 for the k2 / k3 layers
  with >= 64 k rows: B = 12 clips put the down convs' weight gradients there);
* discriminator (C5 widths, B = 2 x 1 s @ 48 kHz, bf16, fwd + bwd incl.
  weight-norm grads): 16 (no prefetching kernels: k_dconv_mfma tiles and the
  generic weight gradient), 25 (scalar bias partials), 28 (128-row tiles for
  the 64-wide grouped convs), 31 (generic VALU kernel for the narrow outputs).

Each variant runs other tiles / reduction orders over the same bf16 operands:
outputs within 1e-2 and gradients within 2e-2 of the default, norm-wise; the
order-only variants (8, 20) must be bit-identical."""
import warnings

import pytest
import torch

pytestmark = pytest.mark.gpu

GEN_KNOBS = [(6, 0xFFFF, False), (7, 0xFFFF, False), (8, 1, True), (12, 0xFFFF, False), (20, 1, True),
             (40, 64, False), (41, 1, True), (56, 1, False), (57, 1, False, 12)]
DISC_KNOBS = [(16, 1, False), (25, 1, False), (28, 1, False), (31, 1, False)]


def _rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30)).item()


def _compare(ref, got, key, exact):
    for i, (r, g) in enumerate(zip(ref, got)):
        if exact:
            assert torch.equal(r, g), (key, i, _rel(g, r))
        else:
            assert _rel(g, r) <= (1e-2 if i == 0 else 2e-2), (key, i, _rel(g, r))


@pytest.mark.parametrize("knob", GEN_KNOBS, ids=[f"key{k[0]}" for k in GEN_KNOBS])
def test_generator_variant_knobs(gpu, knob):
    from models.autoencoder.AudioDec import Generator
    from sel import _lib as Lb
    from sel import configs
    from sel.convops import precision
    key, val, exact = knob[:3]
    B = knob[3] if len(knob) > 3 else 2
    lib = Lb.lib()
    cfg = configs.get("symAD_libritts_24000_hop300")
    torch.manual_seed(3)
    G = Generator(**cfg["generator_params"]).to(gpu)
    G.quantizer.codebook.eval()
    g = torch.Generator(device=gpu).manual_seed(4)
    x = 0.1 * torch.randn(B, 1, 24000, device=gpu, generator=g)
    gy = torch.randn(B, 1, 24000, device=gpu, generator=g)
    params = [p for p in G.parameters() if p.requires_grad]

    def run():
        for p in params:
            p.grad = None
        with precision(torch.bfloat16):
            y, zq, z, vq, _ = G(x)
            ((y * gy).sum() + vq.sum()).backward()
        torch.cuda.synchronize()
        return [y.detach().clone()] + [p.grad.clone() for p in params if p.grad is not None]

    ref = run()
    prev = lib.sel_tune(key, val)
    try:
        got = run()
    finally:
        lib.sel_tune(key, prev)
    assert len(got) == len(ref)
    _compare(ref, got, key, exact)


@pytest.mark.parametrize("knob", DISC_KNOBS, ids=[f"key{k[0]}" for k in DISC_KNOBS])
def test_discriminator_variant_knobs(gpu, knob):
    from models.vocoder.HiFiGAN import Discriminator
    from sel import _lib as Lb
    from sel import configs
    from sel.convops import precision
    key, val, exact = knob[:3]
    B = knob[3] if len(knob) > 3 else 2
    lib = Lb.lib()
    dp = configs.get("symAD_vctk_48000_hop300")["discriminator_params"]
    torch.manual_seed(8)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        D = Discriminator(**dp).to(gpu)
    g = torch.Generator(device=gpu).manual_seed(9)
    x0 = 0.1 * torch.randn(2, 1, 48000, device=gpu, generator=g)
    params = list(D.parameters())

    def run():
        for p in params:
            p.grad = None
        x = x0.clone().requires_grad_(True)
        with precision(torch.bfloat16):
            outs = D(x)
            # every feature map contributes (feature matching) plus the final outputs
            loss = sum((o.float() * (1.0 + 0.01 * j)).mean() for sub in outs for j, o in enumerate(sub))
            loss.backward()
        torch.cuda.synchronize()
        flat = torch.cat([o[-1].detach().float().reshape(-1) for o in outs])
        return [flat, x.grad.clone()] + [p.grad.clone() for p in params]

    ref = run()
    prev = lib.sel_tune(key, val)
    try:
        got = run()
    finally:
        lib.sel_tune(key, prev)
    _compare(ref, got, key, exact)
