"""GPU parity of the step glue: add_noise (dataloader/data_utils.py:12-22), the
split add_noise used under data parallelism, the SNR term
(train_denoise.py:120,140; torchmetrics 1.2.0 formula, parity unpinned beyond
it), and two full train_denoise.py steps (Adam + clip) against the reference's
own run (tests/golden/train_step.npz).

Tolerances: add_noise 1e-6 relative (fp64 norms, fp32 mix); SNR 1e-5 relative
vs the fp64 oracle; the train step as explained in test_train_step_matches_golden.
"""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle import ref_ops as R

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.detach().double().cpu(), torch.as_tensor(b).double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def test_add_noise_matches_reference_golden(gpu):
    from dataloader.data_utils import add_noise
    g = golden("add_noise")
    cl, nz = torch.from_numpy(g["clean"]).to(gpu), torch.from_numpy(g["noise"]).to(gpu)
    for snr in (10, 15, 19):
        out = add_noise(cl, nz, torch.tensor([snr]))
        assert _rel(out, g[f"mixed.{snr}"]) < 1e-6, snr


def test_split_add_noise_equals_fused(gpu):
    from dataloader.data_utils import add_noise
    from sel import dist as D
    torch.manual_seed(0)
    cl = torch.randn(8, 1, 24000, device=gpu)
    nz = 0.3 * torch.randn(8, 1, 24000, device=gpu)
    a = add_noise(cl, nz, 13)
    b = D.add_noise_global(cl, nz, 13)  # world 1: no exchange, same kernels split in two
    assert torch.equal(a, b)
    ref = R.add_noise(cl.double().cpu(), nz.double().cpu(), 13)
    assert _rel(a, ref) < 1e-6


@pytest.mark.parametrize("B,T", [(1, 100), (4, 24000), (64, 24000), (3, 4801)])
def test_snr_fwd_bwd_vs_oracle(gpu, B, T):
    from sel.metrics import SignalNoiseRatio
    torch.manual_seed(B + T)
    t = torch.randn(B, 1, T)
    p = t + 0.3 * torch.randn(B, 1, T)
    pd = p.to(gpu).requires_grad_(True)
    v = SignalNoiseRatio()(pd, t.to(gpu))
    pr = p.double().requires_grad_(True)
    vr = R.snr_db(pr, t.double())
    assert abs(v.item() - vr.item()) <= 1e-5 * abs(vr.item()) + 1e-6
    v.backward(torch.tensor(2.0, device=gpu))
    vr.backward(torch.tensor(2.0, dtype=torch.float64))
    assert _rel(pd.grad, pr.grad) < 1e-5


def test_snr_perfect_prediction_is_finite(gpu):
    from sel.metrics import SignalNoiseRatio
    t = torch.randn(2, 1, 480, device=gpu)
    v = SignalNoiseRatio()(t.clone(), t)
    r = R.snr_db(t.cpu(), t.cpu())  # fp32 inputs -> eps = finfo(float32).eps, as in the reference
    assert torch.isfinite(v) and abs(v.item() - r.item()) < 1e-5 * abs(r.item())


def test_train_step_matches_golden(gpu):
    """Two reference steps (45*mel, backward, clip_grad_norm_(1), Adam(5e-5, wd 1e-6)).

    loss.0 is a forward quantity: 1e-5.  gradnorm: 5e-3 (the log-mel adjoint is
    ill-conditioned; the reference's own fp32 grads are 2.4e-3 from fp64, see
    test_gpu_spectral.cond_close).  Adam's first steps move each weight by about
    +-lr*sign(g), so a weight whose tiny gradient flips sign under that error moves
    2*lr the other way: we bound the FRACTION of such weights (<= 2%) and the
    norm-wise update error (<= 10%), and loss.1 to 1e-4."""
    from models.autoencoder_without_PQC.AudioDec import Generator
    from sel import configs
    from train_denoise import DenoiseStep
    g = golden("train_step")
    gp = dict(encode_channels=4, decode_channels=4, code_dim=64, codebook_num=2, codebook_size=64)
    G = Generator(**gp)
    G.load_state_dict({k[4:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("sd0.")})
    G = G.to(gpu)
    cfg = configs.get("symAD_24Mel")
    step = DenoiseStep(cfg, gpu, generator=G)
    xn, xc = torch.from_numpy(g["x_noisy"]), torch.from_numpy(g["x_clean"])
    lr = cfg["generator_optimizer_params"]["lr"]
    for s in range(2):
        before = {k: v.detach().clone() for k, v in G.named_parameters()}
        loss, _, frags = step.model_step(xc, xn)
        ref_loss = float(g[f"loss.{s}"])
        assert abs(loss.item() - ref_loss) <= (1e-5 if s == 0 else 1e-4) * abs(ref_loss)
        gn = float(g[f"gradnorm.{s}"])
        assert abs(step.last_grad_norm.item() - gn) <= 5e-3 * gn
        flips, tot, num, den = 0, 0, 0.0, 0.0
        for k, p in G.named_parameters():
            ref = torch.from_numpy(g[f"sd{s + 1}.{k}"]).double() - torch.from_numpy(g[f"sd{s}.{k}"]).double()
            d = (p.detach() - before[k]).double().cpu()
            flips += ((d - ref).abs() > 0.5 * lr).sum().item()
            tot += d.numel()
            num += ((d - ref) ** 2).sum().item()
            den += (ref ** 2).sum().item()
            # continue from the reference's weights so step 1 is judged on its own
            with torch.no_grad():
                p.copy_(torch.from_numpy(g[f"sd{s + 1}.{k}"]).to(gpu))
        assert flips <= 0.02 * tot, (s, flips, tot)
        assert (num / den) ** 0.5 <= 0.10, (s, (num / den) ** 0.5)


@pytest.mark.parametrize("bf16", [False, True])
def test_steps_without_copy_use_updated_weights(gpu, bf16):
    """fused Adam writes the parameters without bumping their
    version counters, so the packed conv weights must be refreshed by the
    optimizer step hook.  After three DenoiseStep steps with nothing touching
    the weights in between, the trained generator's forward must equal a fresh
    generator's forward on the same (updated) weights, bit for bit."""
    from models.autoencoder_without_PQC.AudioDec import Generator
    from sel import configs
    from sel.convops import precision
    from train_denoise import DenoiseStep
    gp = dict(encode_channels=8, decode_channels=8, code_dim=64, codebook_num=2, codebook_size=64)
    torch.manual_seed(1)
    G = Generator(**gp).to(gpu)
    cfg = configs.get("symAD_24Mel")
    cfg["generator_optimizer_params"]["lr"] = 1e-3  # visible updates in 3 steps
    step = DenoiseStep(cfg, gpu, generator=G)
    assert step.optimizer["generator"].defaults.get("fused"), "the GPU default is fused Adam"
    g = torch.Generator().manual_seed(2)
    xc = 0.1 * torch.randn(2, 1, 4800, generator=g)
    xn = xc + 0.05 * torch.randn(2, 1, 4800, generator=g)
    dt = torch.bfloat16 if bf16 else torch.float32
    with precision(dt):
        with torch.no_grad():
            y0 = G(xn.to(gpu)).clone()
        for _ in range(3):
            step.model_step(xc, xn)
        with torch.no_grad():
            y1 = G(xn.to(gpu)).clone()
            G2 = Generator(**gp)
            G2.load_state_dict(G.state_dict())
            G2 = G2.to(gpu)
            y2 = G2(xn.to(gpu))
    assert not torch.equal(y0, y1), "the weights did not move"
    assert torch.equal(y1, y2), (y1 - y2).abs().max().item()
