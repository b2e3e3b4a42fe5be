"""Denoising training script — drop-in for the reference's train_denoise.py.

Same CLI (``-e/--environment``, ``-c/--config`` resolved under config/denoise/),
same step semantics (model_step / calculate_generator_loss, :138-263), on the
MI355X path: the without-PQC AudioDec generator (HIP conv primitives), the
fused log-mel L1 loss and the SNR term (HIP kernels), on-device add_noise.

Differences, all outside the numerics of a step:
  * the reference runs at import; here ``main()`` does, and the step logic is a
    reusable ``DenoiseStep`` (bench / tests drive it directly);
  * ClearML logging -> ``ScalarWriter`` (JSON lines under job_out/);
  * environment ``SYNTH``: synthetic 1 s clips, no corpus needed;
  * data parallel: under torchrun (WORLD_SIZE > 1) each rank takes an equal
    shard of the global batch, add_noise uses the global norms
    (sel.dist.add_noise_global) and the SNR term uses the global batch mean
    (see ``_global_snr_term``) — so a DDP step equals the single-device step on
    the global batch;
  * the HiFiGAN discriminator is not built yet: a run whose
    schedule would enable it raises instead of silently training without it.

Reference quirks reproduced on purpose: ``noise_dropout`` runs after mixing and
never changes the model input (:313-319); validation also increments ``steps``
(:384); the "adversarial" term uses the waveform, not discriminator outputs (:147).
"""
import math
import os
import time
from argparse import ArgumentParser

import numpy as np
import torch
from torch import nn

from dataloader.data_utils import add_noise, set_epoch
from losses import MultiMelSpectrogramLoss
from models.autoencoder_without_PQC.AudioDec import Generator as GeneratorAudioDec
from sel import configs as sel_configs
from sel import dist as D
from sel.metrics import SignalNoiseRatio
from trainer.trainerGAN import ScalarWriter


def load_config(path_to_config):
    """YAML file if it exists (yaml.safe_load, as :33-37), else the built-in
    restatement of the named config (sel.configs)."""
    if os.path.exists(path_to_config):
        import yaml
        with open(path_to_config, "r") as f:
            return yaml.safe_load(f)
    name = os.path.splitext(os.path.basename(path_to_config))[0]
    if name in sel_configs.CONFIGS:
        return sel_configs.get(name)
    raise FileNotFoundError(path_to_config)


def _global_snr_term(snr_local, lam):
    """lam * (1 - sigmoid(m)), m = SNR mean over the GLOBAL batch.

    sigmoid(mean) is not a mean over shards, so DDP's gradient averaging alone
    would be wrong.  With m = mean_r m_r (one all-reduce of a scalar), the
    global gradient is -lam*sigmoid'(m) * mean_r dm_r/dtheta; DDP averages the
    per-rank gradients, so each rank back-propagates -lam*sigmoid'(m) * m_r.
    Value: the global term; gradient: exact."""
    if not D.is_dist() or D.rank_world()[1] == 1:
        return lam * (1 - torch.sigmoid(snr_local))
    m = D.allreduce_sum_(snr_local.detach().clone()) / D.rank_world()[1]
    s = torch.sigmoid(m)
    return lam * (1 - s) + (-lam * s * (1 - s)) * (snr_local - snr_local.detach())


class DenoiseStep:
    """model_step + calculate_generator_loss of train_denoise.py:138-263."""

    def __init__(self, config, device, generator=None, optimizer=None, discriminator=None):
        self.config = config
        self.device = device
        self.model = {"generator": generator if generator is not None
                      else GeneratorAudioDec(**config["generator_params"]).to(device),
                      "discriminator": discriminator}
        gen = self.model["generator"]
        # on the GPU: torch's fused multi-tensor Adam (one launch per step, same update rule)
        opt_kw = dict(config["generator_optimizer_params"])
        if next(gen.parameters()).is_cuda:
            opt_kw.setdefault("fused", True)
        self.optimizer = {"generator": optimizer if optimizer is not None
                          else torch.optim.Adam(gen.parameters(), **opt_kw)}
        self.measures = {"MAE": nn.L1Loss(), "SNR": SignalNoiseRatio(),
                         "Mel-loss": MultiMelSpectrogramLoss(**config["mel_loss_params"]).to(device)}
        self.discriminator_enabled = False
        self.last_grad_norm = None  # pre-clip total norm of the last train step (device tensor)

    def train_module(self):
        return self.model["generator"]

    def calculate_generator_loss(self, pred, target):
        c = self.config
        mel_loss = c["lambda_mel_loss"] * self.measures["Mel-loss"](pred, target)
        if c.get("lambda_snr_loss", 0.0):
            snr_loss = _global_snr_term(self.measures["SNR"](pred, target), c["lambda_snr_loss"])
        else:
            # the reference evaluates the SNR term even at weight 0 (value 0 * ...)
            snr_loss = torch.zeros((), device=pred.device)
        if self.discriminator_enabled:
            raise NotImplementedError("HiFiGAN discriminator (SURVEY §8f, row f1) is not built yet")
        zero = torch.zeros((), device=pred.device)
        return mel_loss + snr_loss, (("mel_loss", mel_loss), ("adv_loss", zero), ("feat_loss", zero),
                                     ("snr_loss", snr_loss))

    def model_step(self, target, x, mode="train"):
        gen = self.model["generator"]
        x = x.to(self.device)
        target = target.to(self.device)
        gen.train(mode == "train")
        y_pred = gen(x)
        gen_loss, fragments = self.calculate_generator_loss(y_pred, target)
        if mode == "train":
            opt = self.optimizer["generator"]
            opt.zero_grad()
            gen_loss.backward()
            if self.config["generator_grad_norm"] > 0:
                self.last_grad_norm = torch.nn.utils.clip_grad_norm_(gen.parameters(),
                                                                     self.config["generator_grad_norm"])
            opt.step()
        return gen_loss, torch.zeros((), device=self.device), fragments


def noise_dropout(clean_sample_batch, noise_sample_batch, noise_dropout_rate):
    """:313-319 (result unused by the caller, as in the reference)."""
    for i, clean_sample in enumerate(clean_sample_batch):
        if torch.rand((1,)).item() <= noise_dropout_rate:
            noise_sample_batch[i] = clean_sample
    return noise_sample_batch


def _synthetic_loaders(batch_size, batch_length, n_batches, seed):
    """SURVEY §8d synthetic clips: clean 0.1*N(0,1) (PCG64(seed)), noise PCG64(seed+1)."""
    def gen(s):
        rng = np.random.Generator(np.random.PCG64(s))
        for _ in range(n_batches):
            yield torch.from_numpy((0.1 * rng.standard_normal((batch_size, 1, batch_length))).astype(np.float32))
    return (lambda: gen(seed)), (lambda: gen(seed + 1))


def main(argv=None):
    parser = ArgumentParser()
    parser.add_argument("-e", "--environment", default="LAPTOP")
    parser.add_argument("-c", "--config", default="symAD_custom.yaml")
    parser.add_argument("--synthetic-batches", type=int, default=4, help="SYNTH: batches per epoch")
    parser.add_argument("--epochs", type=int, default=None, help="override config epochs")
    args = parser.parse_args(argv)

    config = load_config(os.path.join("config", "denoise", args.config))
    env = args.environment
    rank, world = D.init_from_env()
    if torch.cuda.is_available():
        device = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
        torch.cuda.set_device(device)
    else:
        raise RuntimeError("train_denoise (MI355X build) needs a ROCm GPU; there is no CPU path")

    SAMPLE_RATE = config["sample_rate"]
    NOISE_DROPOUT_RATE = config["noise_dropout_rate"]
    EPOCHS = args.epochs if args.epochs is not None else config["epochs"]
    if EPOCHS > config["epoch_to_enable_discriminator"]:
        raise NotImplementedError("this schedule enables the HiFiGAN discriminator (SURVEY §8f row f1), "
                                  "not built yet; pass --epochs <= epoch_to_enable_discriminator")
    torch.manual_seed(config["seed"])
    task_name = config.get("experiment_name", "denoise") if env == "HPC" else f"{env}-run"
    writer = ScalarWriter(os.path.join("job_out", task_name) if rank == 0 else None)

    step = DenoiseStep(config, device)
    gen = step.model["generator"]
    if config.get("initial_model", ""):
        ckpt = os.path.join("job_out", config["initial_model"])
        if os.path.exists(ckpt):
            gen.load_state_dict(torch.load(ckpt, map_location=device, weights_only=True))
        else:
            print("No inital model")
    # without-PQC: projector, quantizer and decoder.conv1 never get a gradient
    for mod in (gen.projector, gen.quantizer, gen.decoder.conv1):
        for p in mod.parameters():
            p.requires_grad_(False)
    if world > 1:
        step.model["generator"] = D.wrap_ddp(gen, device)

    batch_length = 1 * SAMPLE_RATE
    batch_size = 4 if env == "LAPTOP" else int(config["batch_size"])
    loaders = ()
    if env == "SYNTH":
        clean_it, noise_it = _synthetic_loaders(batch_size * world, batch_length, args.synthetic_batches,
                                                config["seed"])
        train_pairs = lambda: zip(clean_it(), noise_it())  # noqa: E731
        val_pairs = train_pairs
    else:
        from dataloader.AudioDataset import AudioDataset
        from dataloader.data_utils import get_dataloaders
        paths = {"LAPTOP": ("corpus/train/clean", "clean", "corpus/train/noise", "noise")}
        if env not in paths:
            raise Exception("Illegal argument: " + env)
        cp, cr, npth, nr = paths[env]
        split = [0.7, 0.15, 0.15]
        tc, vc, _ = get_dataloaders(AudioDataset(cp, cr, SAMPLE_RATE), split, batch_size, batch_length,
                                    config["seed"], rank, world)
        tn, vn, _ = get_dataloaders(AudioDataset(npth, nr, SAMPLE_RATE), split, batch_size, batch_length,
                                    config["seed"], rank, world)
        train_pairs = lambda: zip(tc, tn)  # noqa: E731
        val_pairs = lambda: zip(vc, vn)  # noqa: E731
        loaders = (tc, tn, vc, vn)

    def mix(clean, noise):
        snr = torch.randint(10, 20, (1,))
        clean, noise = clean.to(device, non_blocking=True), noise.to(device, non_blocking=True)
        if env == "SYNTH" and world > 1:  # global batch generated on every rank: mix globally, then shard
            return D.shard(clean), D.shard(add_noise(clean, noise, snr))
        if world > 1:
            return clean, D.add_noise_global(clean, noise, snr)
        return clean, add_noise(clean, noise, snr)

    steps = train_steps = config["step"]
    start = time.perf_counter()
    for epoch in range(EPOCHS):
        set_epoch(loaders, epoch)  # data parallel: new shard order every epoch
        if epoch > config["epoch_to_enable_noise_dropout_decay"]:
            NOISE_DROPOUT_RATE -= config["noise_dropout_rate_decay"]
        losses = []
        for i_batch, (clean_batch, noise_batch) in enumerate(train_pairs()):
            if env == "LAPTOP" and i_batch == 3:
                break
            target, mixed = mix(clean_batch, noise_batch)
            if NOISE_DROPOUT_RATE != 0.0:
                noise_batch = noise_dropout(clean_batch, noise_batch, NOISE_DROPOUT_RATE)
            gen_loss, dis_loss, fragments = step.model_step(target, mixed)
            steps += 1
            train_steps += 1
            losses.append(gen_loss.detach())
            if steps % 100 == 0 or env in ("LAPTOP", "SYNTH"):
                writer.add_scalar("Generator Batch Loss/Train", gen_loss.item(), train_steps)
                for name, v in fragments:
                    writer.add_scalar(f"Generator Batch Loss/{name}", float(v), train_steps)
        avg_train = torch.stack(losses).mean().item() if losses else math.nan
        if env == "HPC" and rank == 0:
            os.makedirs("job_out", exist_ok=True)
            torch.save(gen.state_dict(), os.path.join("job_out", f"{task_name}checkpoint-{train_steps}.pkl"))
        val, n = 0.0, 0
        for i_batch, (clean_batch, noise_batch) in enumerate(val_pairs()):
            if env == "LAPTOP" and i_batch == 3:
                break
            target, mixed = mix(clean_batch, noise_batch)
            with torch.no_grad():
                gl, _, _ = step.model_step(target, mixed, mode="eval")
            val += gl.item()
            n += 1
            steps += 1
        writer.add_scalar("Generator Loss/Train", avg_train, epoch)
        writer.add_scalar("Generator Loss/Validation", val / max(n, 1), epoch)
        if rank == 0:
            t = time.perf_counter() - start
            print(f"epoch {epoch}: train {avg_train:.4f} val {val / max(n, 1):.4f} step {train_steps} "
                  f"time {int(t // 3600)}:{int(t // 60 % 60)}:{int(t % 60)}", flush=True)
    return step


if __name__ == "__main__":
    main()
