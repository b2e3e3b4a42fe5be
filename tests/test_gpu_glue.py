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
    """a fused Adam (sel.optim.Adam, or torch's fused kernel)
    writes the parameters without bumping their version counters, so the packed conv weights must be refreshed by the
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
    from sel import optim as O
    opt = step.optimizer["generator"]
    # the GPU default: sel.optim.Adam (raw-pointer update) or torch's fused Adam
    assert isinstance(opt, O.Adam) or opt.defaults.get("fused"), type(opt)
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


def test_denoise_trainer_step_matches_reference_golden(gpu):
    """trainer/denoise.Trainer._train_step (:52-84) against the reference CLASS
    ITSELF run in the build container (tests/golden/trainer_step.npz,
    make_goldens.py --only trainer): reduced-width PQC generator, codebook eval,
    lambda_vq * sum(vqloss) + 45 * mel (libritts-24k mel), decoder/quantizer
    frozen, Adam(1e-4, (0.5, 0.9)) — fused Adam here, two steps with nothing
    touching the weights in between (so the packed-weight refresh is exercised).
    Logged keys and values: mel/vq/generator loss 1e-5 (step 0) / 1e-4 (step 1),
    perplexities 1e-5; updates as in test_train_step_matches_golden."""
    from models.autoencoder.AudioDec import Generator
    from losses import MultiMelSpectrogramLoss
    from trainer.denoise import Trainer
    g = golden("trainer_step")
    gp = dict(encode_channels=4, decode_channels=4, code_dim=64, codebook_num=2, codebook_size=64)
    G = Generator(**gp)
    G.load_state_dict({k[4:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("sd0.")})
    G = G.to(gpu)
    mel = MultiMelSpectrogramLoss(fs=24000, fft_sizes=[2048], hop_sizes=[300], win_lengths=[2048],
                                  window="hann_window", num_mels=80, fmin=0, fmax=12000, log_base=None).to(gpu)
    cfg = {"outdir": None, "train_max_steps": 10, "use_mel_loss": True, "use_stft_loss": False,
           "use_shape_loss": False, "lambda_mel_loss": 45.0, "lambda_vq_loss": 1.0, "generator_grad_norm": -1}
    opt = torch.optim.Adam(G.parameters(), lr=1e-4, betas=(0.5, 0.9), weight_decay=0.0, fused=True)
    sched = torch.optim.lr_scheduler.StepLR(opt, step_size=200000, gamma=1.0)
    tr = Trainer(steps=0, epochs=0, data_loader={}, model={"generator": G, "discriminator": None},
                 criterion={"mel": mel}, optimizer={"generator": opt}, scheduler={"generator": sched},
                 config=cfg, device=gpu)
    xn, xc = torch.from_numpy(g["x_noisy"]), torch.from_numpy(g["x_clean"])
    lr = 1e-4
    trainable = [k for k, p in G.named_parameters() if p.requires_grad]
    assert trainable and all(k.startswith(("encoder.", "projector.")) for k in trainable)
    for s in range(2):
        before = {k: p.detach().clone() for k, p in G.named_parameters()}
        tr._train_step((xn, xc))
        tol = 1e-5 if s == 0 else 1e-4
        rec = {k: float(v) for k, v in tr.total_train_loss.items()}
        ref = {k[len(f"rec.{s}."):]: float(v) for k, v in g.items() if k.startswith(f"rec.{s}.")}
        assert set(rec) == set(ref), set(rec) ^ set(ref)
        for k, v in ref.items():
            assert abs(rec[k] - v) <= tol * abs(v) + 1e-7, (s, k, rec[k], v)
        tr.total_train_loss.clear()
        flips, tot, num, den = 0, 0, 0.0, 0.0
        for k in trainable:
            p = dict(G.named_parameters())[k]
            refd = torch.from_numpy(g[f"sd{s + 1}.{k}"]).double() - (
                torch.from_numpy(g[f"sd{s}.{k}"]).double() if s else before[k].double().cpu())
            d = (p.detach() - before[k]).double().cpu()
            flips += ((d - refd).abs() > 0.5 * lr).sum().item()
            tot += d.numel()
            num += ((d - refd) ** 2).sum().item()
            den += (refd ** 2).sum().item()
        assert flips <= 0.02 * tot, (s, flips, tot)
        assert (num / den) ** 0.5 <= 0.10, (s, (num / den) ** 0.5)
        if s == 0:  # continue from the reference's weights (no version bump: fused Adam + .data)
            for k in trainable:
                with torch.no_grad():
                    dict(G.named_parameters())[k].copy_(torch.from_numpy(g[f"sd1.{k}"]).to(gpu))


@pytest.mark.parametrize("gan", [False, True])
def test_train_denoise_main_synthetic(gpu, tmp_path, monkeypatch, gan):
    """train_denoise.main() end to end under -e SYNTH (synthetic 1 s clips): one
    epoch of training + validation, losses finite and logged; with gan=True a
    reduced config whose schedule enables the discriminator at epoch 0 (GAN step,
    :296-297)."""
    import json
    import train_denoise
    from sel import configs
    monkeypatch.chdir(tmp_path)
    name = "symAD_24Mel"
    if gan:
        c = configs.get("symAD_24Mel")
        c.update(epoch_to_enable_discriminator=0, batch_size=2, lambda_feat_match=2.0,
                 generator_params=dict(c["generator_params"], encode_channels=8, decode_channels=8))
        dp = c["discriminator_params"]
        dp["scale_discriminator_params"] = dict(dp["scale_discriminator_params"], channels=16,
                                                max_downsample_channels=64)
        dp["period_discriminator_params"] = dict(dp["period_discriminator_params"], channels=8,
                                                 max_downsample_channels=64)
        monkeypatch.setitem(configs.CONFIGS, "test_gan", c)
        name = "test_gan"
    step = train_denoise.main(["-e", "SYNTH", "-c", f"{name}.yaml", "--epochs", "1", "--synthetic-batches", "2"])
    assert step.discriminator_enabled == gan
    rows = [json.loads(l) for l in open(tmp_path / "job_out" / "SYNTH-run" / "scalars.jsonl")]
    keys = {r["key"] for r in rows}
    assert {"Generator Batch Loss/Train", "Generator Loss/Validation", "Discriminator Loss/Train"} <= keys
    assert all(np.isfinite(r["value"]) for r in rows)
    dis = [r["value"] for r in rows if r["key"] == "Discriminator Batch Loss/Train"]
    assert (min(dis) > 0) == gan
