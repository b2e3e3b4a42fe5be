"""Denoise fine-tune trainer — drop-in for trainer/denoise.py (Trainer :19-111).

Freezes quantizer + decoder (:43-49), keeps the codebook in eval mode (no EMA,
:60); a step is generator(x_noisy) -> lambda_vq*sum(vqloss) + metric loss vs
x_clean -> _update_generator (:52-84)."""
import logging

import torch

from trainer.trainerGAN import TrainerVQGAN


class Trainer(TrainerVQGAN):
    def __init__(self, steps, epochs, data_loader, model, criterion, optimizer, scheduler, config,
                 device=torch.device("cpu")):
        super().__init__(steps=steps, epochs=epochs, data_loader=data_loader, model=model, criterion=criterion,
                         optimizer=optimizer, scheduler=scheduler, config=config, device=device)
        gen = self.model["generator"]
        gen = getattr(gen, "module", gen)  # DDP-wrapped
        for p in gen.quantizer.parameters():
            p.requires_grad = False
        for p in gen.decoder.parameters():
            p.requires_grad = False
        logging.info("Quantizer, codebook, and decoder are fixed")

    def _gen(self):
        g = self.model["generator"]
        return getattr(g, "module", g)

    def _train_step(self, batch):
        mode = "train"
        x_n, x_c = batch
        x_n = x_n.to(self.device, non_blocking=True)
        x_c = x_c.to(self.device, non_blocking=True)
        self._gen().quantizer.codebook.eval()
        y_nc, zq, z, vqloss, perplexity = self.model["generator"](x_n)
        self._perplexity(perplexity, mode=mode)
        gen_loss = self._vq_loss(vqloss, mode=mode)
        gen_loss = gen_loss + self._metric_loss(y_nc, x_c, mode=mode)
        self._record_loss("generator_loss", gen_loss, mode=mode)
        self._update_generator(gen_loss)
        self.steps += 1
        self.tqdm.update(1)
        self._check_train_finish()

    @torch.no_grad()
    def _eval_step(self, batch):
        mode = "eval"
        x_n, x_c = batch
        x_n = x_n.to(self.device)
        x_c = x_c.to(self.device)
        y_nc, zq, z, vqloss, perplexity = self.model["generator"](x_n)
        self._perplexity(perplexity, mode=mode)
        gen_loss = self._vq_loss(vqloss, mode=mode)
        gen_loss = gen_loss + self._metric_loss(y_nc, x_c, mode=mode)
        self._record_loss("generator_loss", gen_loss, mode=mode)
