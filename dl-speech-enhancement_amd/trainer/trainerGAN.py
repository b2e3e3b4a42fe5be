"""Template GAN training flow — drop-in for trainer/trainerGAN.py (TrainerGAN
:24-347, TrainerVQGAN :350-401).

Same constructor, methods, logged keys (train/mel_loss, train/vqloss,
train/ppl_i, ...) and checkpoint dict layout.  Differences, all behaviour-
preserving: losses are accumulated as device tensors and converted to floats
only when a log interval is written (the reference calls .item() on every loss
of every step, a host sync per loss), and tensorboardX (absent here) is
replaced by a JSON-lines scalar writer with the same add_scalar() call.
"""
import abc
import json
import logging
import os

import torch

try:
    from tqdm import tqdm
except ImportError:  # pragma: no cover
    tqdm = None


class LossTotals(dict):
    """Running loss totals (name -> float or 0-d tensor) like the reference's
    defaultdict(float) + per-step `total[name] += loss.item()`, without a host
    sync and without one tiny add kernel per recorded scalar: device values are
    queued and folded into one accumulator vector (one concatenation + one add
    per flush) when the totals are read or the queue grows."""

    _FLUSH_AT = 256

    def __init__(self):
        super().__init__()
        self._pending = []  # (names, detached tensor with len(names) elements)
        self._acc_names = None
        self._acc = None

    def add(self, name, value):
        if torch.is_tensor(value):
            self.add_vector([name], value)
        else:
            self._materialize()
            dict.__setitem__(self, name, dict.get(self, name, 0.0) + value)

    def add_vector(self, names, value):
        self._pending.append((list(names), value.detach()))
        if len(self._pending) >= self._FLUSH_AT:
            self._flush()

    def _flush(self):
        if not self._pending:
            return
        names = [n for ns, _ in self._pending for n in ns]
        vals = torch.cat([v.reshape(-1).float() for _, v in self._pending])
        self._pending = []
        # entries of one name recorded several times before this flush: fold them
        uniq = list(dict.fromkeys(names))
        if len(uniq) != len(names):
            idx = torch.tensor([uniq.index(n) for n in names], device=vals.device)
            vals = torch.zeros(len(uniq), dtype=vals.dtype, device=vals.device).index_add_(0, idx, vals)
            names = uniq
        if self._acc is not None and self._acc_names == names:
            self._acc += vals
        else:
            self._materialize()
            self._acc_names, self._acc = names, vals

    def _materialize(self):
        self._flush_pending_only()
        if self._acc is None:
            return
        names, acc = self._acc_names, self._acc
        self._acc_names = self._acc = None
        for i, n in enumerate(names):
            dict.__setitem__(self, n, dict.get(self, n, 0.0) + acc[i])

    def _flush_pending_only(self):
        if self._pending:
            pend, self._pending = self._pending, []
            names = [n for ns, _ in pend for n in ns]
            vals = torch.cat([v.reshape(-1).float() for _, v in pend])
            for i, n in enumerate(names):
                dict.__setitem__(self, n, dict.get(self, n, 0.0) + vals[i])

    # reads see every recorded value
    def __getitem__(self, key):
        self._materialize()
        return dict.__getitem__(self, key) if dict.__contains__(self, key) else 0.0

    def __setitem__(self, key, value):
        self._materialize()
        dict.__setitem__(self, key, value)

    def __contains__(self, key):
        self._materialize()
        return dict.__contains__(self, key)

    def keys(self):
        self._materialize()
        return dict.keys(self)

    def items(self):
        self._materialize()
        return dict.items(self)

    def values(self):
        self._materialize()
        return dict.values(self)

    def __iter__(self):
        self._materialize()
        return dict.__iter__(self)

    def __len__(self):
        self._materialize()
        return dict.__len__(self)


class ScalarWriter:
    """add_scalar(key, value, step) -> <outdir>/scalars.jsonl (tensorboardX stand-in)."""

    def __init__(self, outdir):
        self.path = os.path.join(outdir, "scalars.jsonl") if outdir else None
        if self.path:
            os.makedirs(outdir, exist_ok=True)

    def add_scalar(self, key, value, step):
        if self.path:
            with open(self.path, "a") as f:
                f.write(json.dumps({"key": key, "value": float(value), "step": int(step)}) + "\n")


class _NullBar:
    def update(self, n=1):
        pass

    def close(self):
        pass


class TrainerGAN(abc.ABC):
    def __init__(self, steps, epochs, data_loader, model, criterion, optimizer, scheduler, config,
                 device=torch.device("cpu")):
        self.steps = steps
        self.epochs = epochs
        self.data_loader = data_loader
        self.model = model
        self.criterion = criterion
        self.optimizer = optimizer
        self.scheduler = scheduler
        self.config = config
        self.device = device
        self.writer = ScalarWriter(config.get("outdir"))
        self.total_train_loss = LossTotals()
        self.total_eval_loss = LossTotals()
        self.train_max_steps = config.get("train_max_steps", 0)
        self.tqdm = _NullBar()

    @abc.abstractmethod
    def _train_step(self, batch):
        pass

    @abc.abstractmethod
    def _eval_step(self, batch):
        pass

    def run(self):
        self.finish_train = False
        self.tqdm = (tqdm(initial=self.steps, total=self.train_max_steps, desc="[train]")
                     if tqdm is not None else _NullBar())
        while True:
            self._train_epoch()
            if self.finish_train:
                break
        self.tqdm.close()
        logging.info("Finished training.")

    def save_checkpoint(self, checkpoint_path):
        state_dict = {
            "optimizer": {"generator": self.optimizer["generator"].state_dict(),
                          "discriminator": self.optimizer["discriminator"].state_dict()},
            "scheduler": {"generator": self.scheduler["generator"].state_dict(),
                          "discriminator": self.scheduler["discriminator"].state_dict()},
            "steps": self.steps,
            "epochs": self.epochs,
            "model": {"generator": self.model["generator"].state_dict(),
                      "discriminator": self.model["discriminator"].state_dict()},
        }
        d = os.path.dirname(checkpoint_path)
        if d and not os.path.exists(d):
            os.makedirs(d)
        torch.save(state_dict, checkpoint_path)

    def load_checkpoint(self, checkpoint_path, strict=True, load_only_params=False, load_discriminator=True):
        state_dict = torch.load(checkpoint_path, map_location="cpu", weights_only=True)
        self.model["generator"].load_state_dict(state_dict["model"]["generator"], strict=strict)
        self.model["discriminator"].load_state_dict(state_dict["model"]["discriminator"], strict=strict)
        if not load_only_params:
            self.steps = state_dict["steps"]
            self.epochs = state_dict["epochs"]
            self.optimizer["generator"].load_state_dict(state_dict["optimizer"]["generator"])
            self.scheduler["generator"].load_state_dict(state_dict["scheduler"]["generator"])
            if load_discriminator:
                self.optimizer["discriminator"].load_state_dict(state_dict["optimizer"]["discriminator"])
                self.scheduler["discriminator"].load_state_dict(state_dict["scheduler"]["discriminator"])

    def _train_epoch(self):
        train_steps_per_epoch = 0
        for train_steps_per_epoch, batch in enumerate(self.data_loader["train"], 1):
            self._train_step(batch)
            self._check_log_interval()
            self._check_eval_interval()
            self._check_save_interval()
            if self.finish_train:
                return
        self.epochs += 1
        self.train_steps_per_epoch = train_steps_per_epoch
        if train_steps_per_epoch > 200:
            logging.info(f"(Steps: {self.steps}) Finished {self.epochs} epoch training "
                         f"({self.train_steps_per_epoch} steps per epoch).")

    def _eval_epoch(self):
        logging.info(f"(Steps: {self.steps}) Start evaluation.")
        for key in self.model.keys():
            self.model[key].eval()
        eval_steps_per_epoch = 0
        for eval_steps_per_epoch, batch in enumerate(self.data_loader["dev"], 1):
            self._eval_step(batch)
        logging.info(f"(Steps: {self.steps}) Finished evaluation ({eval_steps_per_epoch} steps per epoch).")
        for key in list(self.total_eval_loss.keys()):
            self.total_eval_loss[key] = float(self.total_eval_loss[key]) / max(eval_steps_per_epoch, 1)
            logging.info(f"(Steps: {self.steps}) {key} = {self.total_eval_loss[key]:.4f}.")
        self._write_to_tensorboard(self.total_eval_loss)
        self.total_eval_loss = LossTotals()
        for key in self.model.keys():
            self.model[key].train()

    def _metric_loss(self, predict_y, natural_y, mode="train"):
        """trainerGAN.py:214-241 — mel / multi-resolution STFT / shape losses per use_* flags."""
        # (the running sum starts at the first term: `0.0 + loss` would be one
        # more device kernel per step for an exact no-op)
        metric_loss = 0.0

        def acc(total, term):
            return term if isinstance(total, float) and total == 0.0 else total + term

        if self.config.get("use_mel_loss", False):
            mel_loss = self.criterion["mel"](predict_y, natural_y) * self.config["lambda_mel_loss"]
            self._record_loss("mel_loss", mel_loss, mode=mode)
            metric_loss = acc(metric_loss, mel_loss)
        if self.config.get("use_stft_loss", False):
            sc_loss, mag_loss = self.criterion["stft"](predict_y, natural_y)
            sc_loss = sc_loss * self.config["lambda_stft_loss"]
            mag_loss = mag_loss * self.config["lambda_stft_loss"]
            self._record_loss("spectral_convergence_loss", sc_loss, mode=mode)
            self._record_loss("log_stft_magnitude_loss", mag_loss, mode=mode)
            metric_loss = acc(metric_loss, sc_loss + mag_loss)
        if self.config.get("use_shape_loss", False):
            shape_loss = self.criterion["shape"](predict_y, natural_y) * self.config["lambda_shape_loss"]
            self._record_loss("shape_loss", shape_loss, mode=mode)
            metric_loss = acc(metric_loss, shape_loss)
        return metric_loss

    def _adv_loss(self, predict_p, natural_p=None, mode="train"):
        adv_loss = self.criterion["gen_adv"](predict_p)
        if natural_p is not None:
            fm_loss = self.criterion["feat_match"](predict_p, natural_p)
            self._record_loss("feature_matching_loss", fm_loss, mode=mode)
            adv_loss = adv_loss + self.config["lambda_feat_match"] * fm_loss
        adv_loss = adv_loss * self.config["lambda_adv"]
        self._record_loss("adversarial_loss", adv_loss, mode=mode)
        return adv_loss

    def _dis_loss(self, predict_p, natural_p, mode="train"):
        real_loss, fake_loss = self.criterion["dis_adv"](predict_p, natural_p)
        dis_loss = real_loss + fake_loss
        self._record_loss("real_loss", real_loss, mode=mode)
        self._record_loss("fake_loss", fake_loss, mode=mode)
        self._record_loss("discriminator_loss", dis_loss, mode=mode)
        return dis_loss

    def _update_generator(self, gen_loss):
        """trainerGAN.py:271-281: zero_grad -> backward -> clip (if > 0) -> Adam -> scheduler."""
        self.optimizer["generator"].zero_grad()
        gen_loss.backward()
        if self.config["generator_grad_norm"] > 0:
            torch.nn.utils.clip_grad_norm_(self.model["generator"].parameters(),
                                           self.config["generator_grad_norm"])
        self.optimizer["generator"].step()
        self.scheduler["generator"].step()

    def _update_discriminator(self, dis_loss):
        self.optimizer["discriminator"].zero_grad()
        dis_loss.backward()
        if self.config["discriminator_grad_norm"] > 0:
            torch.nn.utils.clip_grad_norm_(self.model["discriminator"].parameters(),
                                           self.config["discriminator_grad_norm"])
        self.optimizer["discriminator"].step()
        self.scheduler["discriminator"].step()

    def _record_loss(self, name, loss, mode="train"):
        """Accumulate without a host sync; converted to float when written."""
        if mode == "train":
            self.total_train_loss.add(f"train/{name}", loss)
        elif mode == "eval":
            self.total_eval_loss.add(f"eval/{name}", loss)
        else:
            raise NotImplementedError(f"Mode ({mode}) is not supported!")

    def _write_to_tensorboard(self, loss):
        for key, value in loss.items():
            self.writer.add_scalar(key, float(value), self.steps)

    def _check_save_interval(self):
        if self.steps and (self.steps % self.config["save_interval_steps"] == 0):
            self.save_checkpoint(os.path.join(self.config["outdir"], f"checkpoint-{self.steps}steps.pkl"))
            logging.info(f"Successfully saved checkpoint @ {self.steps} steps.")

    def _check_eval_interval(self):
        if self.steps % self.config["eval_interval_steps"] == 0:
            self._eval_epoch()

    def _check_log_interval(self):
        if self.steps % self.config["log_interval_steps"] == 0:
            for key in list(self.total_train_loss.keys()):
                self.total_train_loss[key] = float(self.total_train_loss[key]) / self.config["log_interval_steps"]
                logging.info(f"(Steps: {self.steps}) {key} = {self.total_train_loss[key]:.4f}.")
            self._write_to_tensorboard(self.total_train_loss)
            self.total_train_loss = LossTotals()

    def _check_train_finish(self):
        self.finish_train = self.steps >= self.train_max_steps
        return self.finish_train


class TrainerVQGAN(TrainerGAN):
    def _perplexity(self, perplexity, label=None, mode="train"):
        name = f"{mode}/ppl_{label}" if label else f"{mode}/ppl"
        if mode not in ("train", "eval"):
            raise NotImplementedError(f"Mode ({mode}) is not supported!")
        totals = self.total_train_loss if mode == "train" else self.total_eval_loss
        if torch.numel(perplexity) > 1:
            # one entry per codebook stage (keys {mode}/{name}_{idx}), added as one vector
            totals.add_vector([f"{mode}/{name}_{idx}" for idx in range(torch.numel(perplexity))], perplexity)
        else:
            self._record_loss(name, perplexity, mode=mode)

    def _vq_loss(self, vqloss, label=None, mode="train"):
        name = f"{mode}/vqloss_{label}" if label else f"{mode}/vqloss"
        vqloss = torch.sum(vqloss) * self.config["lambda_vq_loss"]
        self._record_loss(name, vqloss, mode=mode)
        return vqloss
