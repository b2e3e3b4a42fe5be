"""Feature matching loss — drop-in for the reference ``losses/feat_match_loss.py``
(FeatureMatchLoss :13-55).  Each per-layer L1 is a HIP reduction over the
feature-map views (sel.dconvops.l1_mean); its gradient is written in the
discriminator buffer's own layout, which the discriminator backward consumes
in place."""
import os

import torch

from sel import dconvops as DC

# SEL_FM_STACK=0: the reference's per-term add / divide accumulation
_STACKED = os.environ.get("SEL_FM_STACK", "1") != "0"


class FeatureMatchLoss(torch.nn.Module):
    """Feature matching loss module."""

    def __init__(self, average_by_layers=True, average_by_discriminators=True, include_final_outputs=False):
        super().__init__()
        self.average_by_layers = average_by_layers
        self.average_by_discriminators = average_by_discriminators
        self.include_final_outputs = include_final_outputs

    def forward(self, feats_hat, feats):
        if not _STACKED:
            return self._forward_loop(feats_hat, feats)
        # sum_i [ sum_j mean|h_ij - f_ij| / J_i ] / I  (feat_match_loss.py:37-55), with
        # each term's 1/J_i and 1/I folded into its reduction kernel's scale and the
        # terms summed by one stack + sum instead of one add (and divide) per term
        pairs = list(zip(feats_hat, feats))
        n_d = len(pairs)
        terms = []
        for feats_hat_, feats_ in pairs:
            if not self.include_final_outputs:
                feats_hat_ = feats_hat_[:-1]
                feats_ = feats_[:-1]
            n_l = min(len(feats_hat_), len(feats_))
            if n_l == 0:
                continue
            w = (1.0 / n_l if self.average_by_layers else 1.0) * (1.0 / n_d if self.average_by_discriminators else 1.0)
            for feat_hat_, feat_ in zip(feats_hat_, feats_):
                terms.append(DC.l1_mean(feat_hat_, feat_.detach(), w))
        if not terms:
            return 0.0
        return torch.stack(terms).sum()

    def _forward_loop(self, feats_hat, feats):
        """The reference's accumulation order, one add / divide per term (SEL_FM_STACK=0)."""
        feat_match_loss = 0.0
        for i, (feats_hat_, feats_) in enumerate(zip(feats_hat, feats)):
            feat_match_loss_ = 0.0
            if not self.include_final_outputs:
                feats_hat_ = feats_hat_[:-1]
                feats_ = feats_[:-1]
            for j, (feat_hat_, feat_) in enumerate(zip(feats_hat_, feats_)):
                feat_match_loss_ = feat_match_loss_ + DC.l1_mean(feat_hat_, feat_.detach())
            if self.average_by_layers:
                feat_match_loss_ = feat_match_loss_ / (j + 1)
            feat_match_loss = feat_match_loss + feat_match_loss_
        if self.average_by_discriminators:
            feat_match_loss = feat_match_loss / (i + 1)
        return feat_match_loss
