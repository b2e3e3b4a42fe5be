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
  * GAN mode (epoch >= epoch_to_enable_discriminator): the HiFi-GAN MSD + MPD
    discriminator runs on the HIP discriminator kernels; the discriminator step
    scores D(target) and D(pred) as one batch (one backward), its real half
    taken from the generator step's D(target) (same weights, same clips) in a
    single process.

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
from losses import (DiscriminatorAdversarialLoss, FeatureMatchLoss, GeneratorAdversarialLoss,
                    MultiMelSpectrogramLoss)
from models.autoencoder_without_PQC.AudioDec import Generator as GeneratorAudioDec
from models.vocoder.HiFiGAN import Discriminator as DiscriminatorHiFiGAN
from models.vocoder.modules.discriminator import frozen_parameters
from sel import configs as sel_configs
from sel import dist as D
from sel import optim as sel_optim
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


def _unwrap(m):
    return getattr(m, "module", m)


class DenoiseStep:
    """model_step + calculate_generator_loss / calculate_discriminator_loss of
    train_denoise.py:138-165, :213-263 (GAN mode once ``discriminator_enabled``)."""

    def __init__(self, config, device, generator=None, optimizer=None, discriminator=None,
                 disc_optimizer=None):
        self.config = config
        self.device = device
        self.model = {"generator": generator if generator is not None
                      else GeneratorAudioDec(**config["generator_params"]).to(device),
                      "discriminator": discriminator}
        gen = self.model["generator"]
        on_gpu = next(gen.parameters()).is_cuda
        # on the GPU: sel.optim.Adam (every tensor's update in one launch; SEL_ADAM=torch:
        # torch's fused multi-tensor Adam), the same update rule and state layout
        opt_kw = dict(config["generator_optimizer_params"])
        if on_gpu:
            opt_kw.setdefault("fused", True)
        self.optimizer = {"generator": optimizer if optimizer is not None
                          else sel_optim.adam(gen.parameters(), **opt_kw)}
        if discriminator is not None:
            dkw = dict(config.get("discriminator_optimizer_params", {}))
            if on_gpu:
                dkw.setdefault("fused", True)
            self.optimizer["discriminator"] = (disc_optimizer if disc_optimizer is not None
                                               else sel_optim.adam(discriminator.parameters(), **dkw))
            self._d_opt_steps = 0

            def _d_stepped(*_):
                self._d_opt_steps += 1
            self.optimizer["discriminator"].register_step_post_hook(_d_stepped)
        self.measures = {"MAE": nn.L1Loss(), "SNR": SignalNoiseRatio(),
                         "Mel-loss": MultiMelSpectrogramLoss(**config["mel_loss_params"]).to(device)}
        # :123-131 (note: FeatureMatchLoss() with its DEFAULT averaging, as the reference builds it)
        self.criterion = {"gen_adv": GeneratorAdversarialLoss(**config.get("generator_adv_loss_params", {})),
                          "dis_adv": DiscriminatorAdversarialLoss(**config.get("discriminator_adv_loss_params", {})),
                          "feat_match": FeatureMatchLoss()}
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
        zero = torch.zeros((), device=pred.device)
        adv_loss = feat_loss = zero
        if self.discriminator_enabled:
            # D only carries the gradient to the generator here (its own grads
            # are discarded by the D step's zero_grad): constant parameters, and
            # the unwrapped module so no DDP reducer waits for them
            Dm = _unwrap(self.model["discriminator"])
            with frozen_parameters(Dm) as D:
                p_ = D(pred)
            self._drop_stash()
            if self._reuse_real():
                # D(target) is also the real half of the D step (:160): D's weights
                # change only in that step's Adam update.  Computed once, into the
                # D step's buffers (Discriminator.stash_first_half); valid for
                # exactly this target tensor and these D parameters (_stash_key)
                p = Dm.stash_first_half(target)
                self._stashed = self._stash_key(target)
            else:
                with torch.no_grad():
                    p = Dm(target)
            adv_loss = c["lambda_adv"] * self.criterion["gen_adv"](pred)  # :147 passes the waveform (quirk)
            feat_loss = c["lambda_feat_match"] * self.criterion["feat_match"](p_, p)
        return mel_loss + adv_loss + feat_loss + snr_loss, (("mel_loss", mel_loss), ("adv_loss", adv_loss),
                                                            ("feat_loss", feat_loss), ("snr_loss", snr_loss))

    def calculate_discriminator_loss(self, pred, target):
        """:157-165, with D(target) and D(pred) as ONE pass over the concatenated
        batch (every clip is independent: identical outputs, one backward per
        forward under DDP)."""
        D = self.model["discriminator"]
        B = target.shape[0]
        st = getattr(self, "_stashed", None)
        if st is not None and st[0] is target and st[1:] == self._stash_key(target)[1:]:
            # the real half was computed in the generator step from this same
            # target and the same D weights: only D(pred) runs
            self._stashed = None
            outs = _unwrap(D).forward_second_half(pred)
        else:
            self._drop_stash()
            outs = D(torch.cat([target, pred], 0))
        p = [[t[:B] for t in o] for o in outs]
        p_ = [[t[B:] for t in o] for o in outs]
        real_loss, fake_loss = self.criterion["dis_adv"](p_, p)
        return (real_loss + fake_loss) * self.config["lambda_adv"]

    def _stash_key(self, target):
        """What a stashed D(target) is valid for: the target tensor itself (and
        its version), the D parameters' versions and the D optimizer's step count
        (torch's fused Adam writes the parameters without bumping _version)."""
        Dm = _unwrap(self.model["discriminator"])
        return (target, target._version, tuple(p._version for p in Dm.parameters()),
                getattr(self, "_d_opt_steps", 0))

    def _drop_stash(self):
        """Forget a stashed real half (and free its 2B-clip buffers)."""
        self._stashed = None
        Dm = _unwrap(self.model["discriminator"]) if self.model.get("discriminator") is not None else None
        if Dm is not None and hasattr(Dm, "clear_stash"):
            Dm.clear_stash()

    def _reuse_real(self):
        """Reuse the generator step's D(target) as the D step's real half: one
        process only (under DDP the D step stays ONE module call over the
        concatenated batch, for the reducer's hooks); SEL_REUSE_REAL=0: off."""
        return (os.environ.get("SEL_REUSE_REAL", "1") != "0" and not (D.is_dist() and D.rank_world()[1] > 1)
                and hasattr(_unwrap(self.model["discriminator"]), "stash_first_half"))

    def model_step(self, target, x, mode="train"):
        gen = self.model["generator"]
        x = x.to(self.device)
        target = target.to(self.device)
        gen.train(mode == "train")
        if self.discriminator_enabled:
            self.model["discriminator"].train(mode == "train")
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
        dis_loss = torch.zeros((), device=self.device)
        if self.discriminator_enabled:
            with torch.no_grad():
                y_pred = gen(x)
            dis_loss = self.calculate_discriminator_loss(y_pred.detach(), target)
            if mode == "train":
                od = self.optimizer["discriminator"]
                od.zero_grad()
                dis_loss.backward()
                if self.config["discriminator_grad_norm"] > 0:
                    torch.nn.utils.clip_grad_norm_(self.model["discriminator"].parameters(),
                                                   self.config["discriminator_grad_norm"])
                od.step()
        return gen_loss, dis_loss, fragments


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


# :47-67.  HPC corpus locations default to the reference's and can be moved
# with SEL_HPC_CLEAN_PATH / SEL_HPC_NOISE_PATH (the roots are the directory names).
ENV_PATHS = {
    "LAPTOP": ("corpus/train/clean", "clean", "corpus/train/noise", "noise"),
    "HPC": (os.environ.get("SEL_HPC_CLEAN_PATH", "/work3/s164396/data/DNS-Challenge-4/datasets_fullband/"
                                                 "clean_fullband/vctk_wav48_silence_trimmed"),
            "vctk_wav48_silence_trimmed",
            os.environ.get("SEL_HPC_NOISE_PATH", "/work3/s164396/data/DNS-Challenge-4/datasets_fullband/"
                                                 "noise_fullband"),
            "noise_fullband"),
}


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
    if env not in ENV_PATHS and env != "SYNTH":
        raise Exception("Illegal argument: " + env)
    torch.manual_seed(config["seed"])
    task_name = config.get("experiment_name", "denoise") if env == "HPC" else f"{env}-run"
    writer = ScalarWriter(os.path.join("job_out", task_name) if rank == 0 else None)

    disc = None
    if config.get("discriminator_params") is not None:  # :97-98 (built always, enabled by the schedule)
        disc = DiscriminatorHiFiGAN(**config["discriminator_params"]).to(device)
    step = DenoiseStep(config, device, discriminator=disc)
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
        if disc is not None:
            step.model["discriminator"] = D.wrap_ddp(disc, device)

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
        cp, cr, npth, nr = ENV_PATHS[env]
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
        if disc is not None and epoch == config["epoch_to_enable_discriminator"]:  # :296-297
            step.discriminator_enabled = True
        if epoch > config["epoch_to_enable_noise_dropout_decay"]:
            NOISE_DROPOUT_RATE -= config["noise_dropout_rate_decay"]
        losses, dlosses = [], []
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
            dlosses.append(dis_loss.detach())
            if steps % 100 == 0 or env in ("LAPTOP", "SYNTH"):
                writer.add_scalar("Generator Batch Loss/Train", gen_loss.item(), train_steps)
                writer.add_scalar("Discriminator Batch Loss/Train", dis_loss.item(), train_steps)
                for name, v in fragments:
                    writer.add_scalar(f"Generator Batch Loss/{name}", float(v), train_steps)
        avg_train = torch.stack(losses).mean().item() if losses else math.nan
        avg_dtrain = torch.stack(dlosses).mean().item() if dlosses else math.nan
        if env == "HPC" and rank == 0:
            os.makedirs("job_out", exist_ok=True)
            torch.save(gen.state_dict(), os.path.join("job_out", f"{task_name}checkpoint-{train_steps}.pkl"))
        val, dval, n = 0.0, 0.0, 0
        for i_batch, (clean_batch, noise_batch) in enumerate(val_pairs()):
            if env == "LAPTOP" and i_batch == 3:
                break
            target, mixed = mix(clean_batch, noise_batch)
            with torch.no_grad():
                gl, dl, _ = step.model_step(target, mixed, mode="eval")
            val += gl.item()
            dval += dl.item()
            n += 1
            steps += 1
        writer.add_scalar("Generator Loss/Train", avg_train, epoch)
        writer.add_scalar("Generator Loss/Validation", val / max(n, 1), epoch)
        writer.add_scalar("Discriminator Loss/Train", avg_dtrain, epoch)
        writer.add_scalar("Discriminator Loss/Validation", dval / max(n, 1), epoch)
        if rank == 0:
            t = time.perf_counter() - start
            print(f"epoch {epoch}: train {avg_train:.4f} val {val / max(n, 1):.4f} step {train_steps} "
                  f"time {int(t // 3600)}:{int(t // 60 % 60)}:{int(t % 60)}", flush=True)
    return step


if __name__ == "__main__":
    main()
