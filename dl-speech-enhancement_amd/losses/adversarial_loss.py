"""Adversarial losses — drop-in for the reference ``losses/adversarial_loss.py``
(GeneratorAdversarialLoss :13-58, DiscriminatorAdversarialLoss :61-124).

Same constructor arguments and return values; each per-discriminator term is a
HIP reduction over the (strided) output view (sel.dconvops.GanReduceFn):
LSGAN ``mse(x, 1)`` / ``mse(x, 0)`` or the hinge terms."""
import torch

from sel import dconvops as DC


class GeneratorAdversarialLoss(torch.nn.Module):
    """Generator adversarial loss module."""

    def __init__(self, average_by_discriminators=True, loss_type="mse"):
        super().__init__()
        self.average_by_discriminators = average_by_discriminators
        assert loss_type in ["mse", "hinge"], f"{loss_type} is not supported."
        self.criterion = self._mse_loss if loss_type == "mse" else self._hinge_loss

    def forward(self, outputs):
        if isinstance(outputs, (tuple, list)):
            adv_loss = 0.0
            for i, outputs_ in enumerate(outputs):
                if isinstance(outputs_, (tuple, list)):
                    outputs_ = outputs_[-1]  # case including feature maps
                adv_loss = adv_loss + self.criterion(outputs_)
            if self.average_by_discriminators:
                adv_loss = adv_loss / (i + 1)
        else:
            adv_loss = self.criterion(outputs)
        return adv_loss

    def _mse_loss(self, x):
        return DC.mse_to(x, 1.0)

    def _hinge_loss(self, x):
        return DC.neg_mean(x)


class DiscriminatorAdversarialLoss(torch.nn.Module):
    """Discriminator adversarial loss module."""

    def __init__(self, average_by_discriminators=True, loss_type="mse"):
        super().__init__()
        self.average_by_discriminators = average_by_discriminators
        assert loss_type in ["mse", "hinge"], f"{loss_type} is not supported."
        if loss_type == "mse":
            self.fake_criterion = self._mse_fake_loss
            self.real_criterion = self._mse_real_loss
        else:
            self.fake_criterion = self._hinge_fake_loss
            self.real_criterion = self._hinge_real_loss

    def forward(self, outputs_hat, outputs):
        if isinstance(outputs, (tuple, list)):
            real_loss = 0.0
            fake_loss = 0.0
            for i, (outputs_hat_, outputs_) in enumerate(zip(outputs_hat, outputs)):
                if isinstance(outputs_hat_, (tuple, list)):
                    outputs_hat_ = outputs_hat_[-1]
                    outputs_ = outputs_[-1]
                real_loss = real_loss + self.real_criterion(outputs_)
                fake_loss = fake_loss + self.fake_criterion(outputs_hat_)
            if self.average_by_discriminators:
                fake_loss = fake_loss / (i + 1)
                real_loss = real_loss / (i + 1)
        else:
            real_loss = self.real_criterion(outputs)
            fake_loss = self.fake_criterion(outputs_hat)
        return real_loss, fake_loss

    def _mse_real_loss(self, x):
        return DC.mse_to(x, 1.0)

    def _mse_fake_loss(self, x):
        return DC.mse_to(x, 0.0)

    def _hinge_real_loss(self, x):
        return DC.hinge(x, real=True)

    def _hinge_fake_loss(self, x):
        return DC.hinge(x, real=False)
