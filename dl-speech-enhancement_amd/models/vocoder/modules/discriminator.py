"""HiFi-GAN discriminators — drop-in for the reference
``models/vocoder/modules/discriminator.py`` (:26-447).

Same classes, constructor arguments, sub-module names and ``state_dict`` keys:
the parameters live in torch ``Conv1d`` / ``Conv2d`` modules built exactly as in
the reference (same init order, ``torch.nn.utils.weight_norm`` on the Conv2d of
the period discriminators -> ``weight_g`` / ``weight_v``), so reference
checkpoints load unchanged.  ``forward`` never calls those modules: each
sub-discriminator runs as one HIP chain (sel/dconvops.ChainFn) in the active
precision (sel.convops.precision) and returns the reference-layout views of its
per-layer outputs.

Reference quirk kept: ``apply_weight_norm`` / ``apply_spectral_norm`` of the
SCALE discriminator only match ``Conv2d`` (:354-372), so the MSD is never
normalised — whatever ``follow_official_norm`` says.
"""
import contextlib
import copy
import logging

import torch
import torch.nn as nn
from torch.nn.utils.spectral_norm import SpectralNorm

from sel import convops as CO
from sel import dconvops as DC


def _slope(name, params):
    if name != "LeakyReLU":
        raise NotImplementedError(f"discriminator activation {name}: only LeakyReLU is lowered to the HIP path")
    return float(params.get("negative_slope", 0.01))


@contextlib.contextmanager
def frozen_parameters(module):
    """Run a discriminator with its parameters as constants (no weight-gradient
    kernels; the parameters receive no gradient and fire no DDP hook).  train_denoise.py's generator step back-propagates through D only
    to reach the generator; the D gradients it also computes (:234-235) are
    discarded by optimizer["discriminator"].zero_grad() before the D step
    (:252), so skipping them changes no result."""
    subs = [m for m in module.modules() if hasattr(m, "_params")]
    prev = [getattr(m, "_frozen", False) for m in subs]
    for m in subs:
        m._frozen = True
    try:
        yield module
    finally:
        for m, p in zip(subs, prev):
            m._frozen = p


class HiFiGANPeriodDiscriminator(nn.Module):
    """HiFiGAN period discriminator module (discriminator.py:26-157)."""

    def __init__(self, in_channels=1, out_channels=1, period=3, kernel_sizes=[5, 3], channels=32,
                 downsample_scales=[3, 3, 3, 3, 1], max_downsample_channels=1024, bias=True,
                 nonlinear_activation="LeakyReLU", nonlinear_activation_params={"negative_slope": 0.1},
                 use_weight_norm=True, use_spectral_norm=False):
        super().__init__()
        assert len(kernel_sizes) == 2
        assert kernel_sizes[0] % 2 == 1, "Kernel size must be odd number."
        assert kernel_sizes[1] % 2 == 1, "Kernel size must be odd number."
        self.period = period
        self.slope = _slope(nonlinear_activation, nonlinear_activation_params)
        self.convs = nn.ModuleList()
        in_chs, out_chs = in_channels, channels
        self._specs = []
        for downsample_scale in downsample_scales:
            self.convs += [nn.Sequential(
                nn.Conv2d(in_chs, out_chs, (kernel_sizes[0], 1), (downsample_scale, 1),
                          padding=((kernel_sizes[0] - 1) // 2, 0)),
                getattr(nn, nonlinear_activation)(**nonlinear_activation_params))]
            self._specs.append((in_chs, out_chs, kernel_sizes[0], downsample_scale, (kernel_sizes[0] - 1) // 2, 1,
                                True))
            in_chs = out_chs
            out_chs = min(out_chs * 4, max_downsample_channels)
        self.output_conv = nn.Conv2d(out_chs, out_channels, (kernel_sizes[1] - 1, 1), 1,
                                     padding=((kernel_sizes[1] - 1) // 2, 0))
        self._specs.append((out_chs, out_channels, kernel_sizes[1] - 1, 1, (kernel_sizes[1] - 1) // 2, 1, False))
        if use_weight_norm and use_spectral_norm:
            raise ValueError("Either use use_weight_norm or use_spectral_norm.")
        self.use_weight_norm = use_weight_norm
        if use_weight_norm:
            self.apply_weight_norm()
        if use_spectral_norm:
            self.apply_spectral_norm()
        self._plan = None

    def _convs(self):
        return [seq[0] for seq in self.convs] + [self.output_conv]

    def _params(self, power=None):
        """The chain's parameter list.  Spectral-normalised convs contribute
        weight_orig / sigma (torch.nn.utils.spectral_norm's own compute_weight,
        i.e. what the reference's module pre-hook sets before each call, with
        its power iteration when the module is training; power=False: reuse
        the current u, v — the second half of a stashed forward)."""
        out = []
        for m in self._convs():
            if self.use_weight_norm:
                out += [m.weight_v, m.weight_g, m.bias]
            else:
                sn = _spectral_norm_hook(m)
                w = m.weight if sn is None else sn.compute_weight(
                    m, do_power_iteration=m.training if power is None else power)
                out += [w, m.bias]
        return out

    def plan(self):
        if self._plan is None:
            self._plan = [DC.LayerSpec(*s) for s in self._specs]
        return self._plan

    def _x0(self, x):
        """(B, 1, T) -> folded sequences (B*p, L_alloc, 1) in the compute dtype, L_valid."""
        b, c, t = x.shape
        if c != 1:
            raise NotImplementedError("the HIP period discriminator takes 1-channel input (in_channels=1)")
        p = self.period
        Lv = (t + p - 1) // p
        seqs = DC.MpdFoldFn.apply(x.reshape(b, t).float(), p, DC.period_alloc(Lv, self.plan()))
        return CO.cast(seqs, CO.compute_dtype()).unsqueeze(-1), Lv

    def _outs(self, views):
        outs = list(views)
        outs[-1] = torch.flatten(outs[-1], 1, -1)
        return outs

    def forward(self, x):
        """x (B, in_channels, T) -> list of each layer's output (B, C, T/p, p), the
        last flattened to (B, T'/p * p) (discriminator.py:110-137)."""
        x0, Lv = self._x0(x)
        return self._outs(DC.ChainFn.apply(x0, Lv, self.plan(), self.slope, self.use_weight_norm, "period",
                                           x.shape[0], self.period, getattr(self, "_frozen", False), None,
                                           *self._params()))

    @torch.no_grad()
    def stash_first_half(self, x):
        """forward(x) of B clips into buffers sized for 2B (the first half),
        kept for forward_second_half; returns the B clips' outputs (no graph)."""
        x0h, Lv = self._x0(x)
        n = x0h.shape[0]
        x0 = torch.empty((2 * n,) + tuple(x0h.shape[1:]), dtype=x0h.dtype, device=x0h.device)
        x0[:n] = x0h
        bufs, geo = DC.chain_forward(x0, Lv, self.plan(), self.slope, self.use_weight_norm, self._params(), 0, n)
        self._stash = (x0, bufs, n, Lv)
        b = x.shape[0]
        return self._outs(DC._view(y[:n], "period", b, g[2], self.period) for y, g in zip(bufs, geo))

    def forward_second_half(self, x):
        """forward(cat[stashed clips, x]) with the stashed half not recomputed."""
        x0, bufs, n, Lv = _take_stash(self)
        x0[n:] = self._x0(x)[0].detach()
        # (spectral norm: stash_first_half ran this call's power iteration)
        return self._outs(DC.ChainFn.apply(x0, Lv, self.plan(), self.slope, self.use_weight_norm, "period",
                                           2 * x.shape[0], self.period, getattr(self, "_frozen", False),
                                           (n, bufs), *self._params(power=False)))

    def apply_weight_norm(self):
        def _apply_weight_norm(m):
            if isinstance(m, nn.Conv2d):
                nn.utils.weight_norm(m)
                logging.debug(f"Weight norm is applied to {m}.")
        self.apply(_apply_weight_norm)

    def apply_spectral_norm(self):
        """discriminator.py:150-157: torch.nn.utils.spectral_norm on every Conv2d
        (weight_orig / weight_u / weight_v, as in the reference's state_dict)."""
        def _apply_spectral_norm(m):
            if isinstance(m, nn.Conv2d):
                nn.utils.spectral_norm(m)
                logging.debug(f"Spectral norm is applied to {m}.")
        self.apply(_apply_spectral_norm)


def _spectral_norm_hook(m):
    for h in m._forward_pre_hooks.values():
        if isinstance(h, SpectralNorm):
            return h
    return None


def _take_stash(f):
    """The stash_first_half state of sub-discriminator f, consumed (a clear error
    instead of an unpacking failure when there is none)."""
    st = getattr(f, "_stash", None)
    if st is None:
        raise RuntimeError(f"{type(f).__name__}.forward_second_half needs a stash_first_half of the same step")
    f._stash = None
    return st


class HiFiGANMultiPeriodDiscriminator(nn.Module):
    """HiFiGAN multi-period discriminator module (discriminator.py:160-209)."""

    def __init__(self, periods=[2, 3, 5, 7, 11],
                 discriminator_params={"in_channels": 1, "out_channels": 1, "kernel_sizes": [5, 3], "channels": 32,
                                       "downsample_scales": [3, 3, 3, 3, 1], "max_downsample_channels": 1024,
                                       "bias": True, "nonlinear_activation": "LeakyReLU",
                                       "nonlinear_activation_params": {"negative_slope": 0.1},
                                       "use_weight_norm": True, "use_spectral_norm": False}):
        super().__init__()
        self.discriminators = nn.ModuleList()
        for period in periods:
            params = copy.deepcopy(discriminator_params)
            params["period"] = period
            self.discriminators += [HiFiGANPeriodDiscriminator(**params)]

    def forward(self, x):
        return [f(x) for f in self.discriminators]

    def stash_first_half(self, x):
        return [f.stash_first_half(x) for f in self.discriminators]

    def forward_second_half(self, x):
        return [f.forward_second_half(x) for f in self.discriminators]


class HiFiGANScaleDiscriminator(nn.Module):
    """HiFi-GAN scale discriminator module (discriminator.py:212-372)."""

    def __init__(self, in_channels=1, out_channels=1, kernel_sizes=[15, 41, 5, 3], channels=128,
                 max_downsample_channels=1024, max_groups=16, bias=True, downsample_scales=[2, 2, 4, 4, 1],
                 nonlinear_activation="LeakyReLU", nonlinear_activation_params={"negative_slope": 0.1},
                 use_weight_norm=True, use_spectral_norm=False):
        super().__init__()
        self.layers = nn.ModuleList()
        assert len(kernel_sizes) == 4
        for ks in kernel_sizes:
            assert ks % 2 == 1
        self.slope = _slope(nonlinear_activation, nonlinear_activation_params)
        self._specs = []
        self.layers += [nn.Sequential(
            nn.Conv1d(in_channels, channels, kernel_sizes[0], bias=bias, padding=(kernel_sizes[0] - 1) // 2),
            getattr(nn, nonlinear_activation)(**nonlinear_activation_params))]
        self._specs.append((in_channels, channels, kernel_sizes[0], 1, (kernel_sizes[0] - 1) // 2, 1, True))
        in_chs, out_chs, groups = channels, channels, 4
        for downsample_scale in downsample_scales:
            self.layers += [nn.Sequential(
                nn.Conv1d(in_chs, out_chs, kernel_size=kernel_sizes[1], stride=downsample_scale,
                          padding=(kernel_sizes[1] - 1) // 2, groups=groups, bias=bias),
                getattr(nn, nonlinear_activation)(**nonlinear_activation_params))]
            self._specs.append((in_chs, out_chs, kernel_sizes[1], downsample_scale, (kernel_sizes[1] - 1) // 2,
                                groups, True))
            in_chs = out_chs
            out_chs = min(in_chs * 2, max_downsample_channels)
            groups = min(groups * 4, max_groups)
        out_chs = min(in_chs * 2, max_downsample_channels)
        self.layers += [nn.Sequential(
            nn.Conv1d(in_chs, out_chs, kernel_size=kernel_sizes[2], stride=1, padding=(kernel_sizes[2] - 1) // 2,
                      bias=bias),
            getattr(nn, nonlinear_activation)(**nonlinear_activation_params))]
        self._specs.append((in_chs, out_chs, kernel_sizes[2], 1, (kernel_sizes[2] - 1) // 2, 1, True))
        self.layers += [nn.Conv1d(out_chs, out_channels, kernel_size=kernel_sizes[3], stride=1,
                                  padding=(kernel_sizes[3] - 1) // 2, bias=bias)]
        self._specs.append((out_chs, out_channels, kernel_sizes[3], 1, (kernel_sizes[3] - 1) // 2, 1, False))
        if use_weight_norm and use_spectral_norm:
            raise ValueError("Either use use_weight_norm or use_spectral_norm.")
        # reference: both only touch Conv2d -> no-ops for this Conv1d stack (:354-372)
        self._plan = None
        self._bias = bias

    def _convs(self):
        return [l[0] if isinstance(l, nn.Sequential) else l for l in self.layers]

    def _params(self):
        out = []
        for m in self._convs():
            out += [m.weight, m.bias]
        return out

    def plan(self):
        if self._plan is None:
            self._plan = [DC.LayerSpec(*s) for s in self._specs]
        return self._plan

    def _x0(self, x):
        b, c, t = x.shape
        if c != 1:
            raise NotImplementedError("the HIP scale discriminator takes 1-channel input (in_channels=1)")
        return CO.cast(x.reshape(b, t, 1).float(), CO.compute_dtype())

    def forward(self, x):
        """x (B, 1, T) -> list of each layer's output (B, C, T_l) (:337-352)."""
        return list(DC.ChainFn.apply(self._x0(x), x.shape[2], self.plan(), self.slope, False, "scale", x.shape[0],
                                     1, getattr(self, "_frozen", False), None, *self._params()))

    @torch.no_grad()
    def stash_first_half(self, x):
        """as HiFiGANPeriodDiscriminator.stash_first_half"""
        x0h = self._x0(x)
        b, t = x.shape[0], x.shape[2]
        x0 = torch.empty((2 * b,) + tuple(x0h.shape[1:]), dtype=x0h.dtype, device=x0h.device)
        x0[:b] = x0h
        bufs, geo = DC.chain_forward(x0, t, self.plan(), self.slope, False, self._params(), 0, b)
        self._stash = (x0, bufs, b, t)
        return [DC._view(y[:b], "scale", b, g[2], 1) for y, g in zip(bufs, geo)]

    def forward_second_half(self, x):
        x0, bufs, b, t = _take_stash(self)
        x0[b:] = self._x0(x).detach()
        return list(DC.ChainFn.apply(x0, t, self.plan(), self.slope, False, "scale", 2 * b, 1,
                                     getattr(self, "_frozen", False), (b, bufs), *self._params()))

    def apply_weight_norm(self):
        pass  # reference :354-362 matches Conv2d only

    def apply_spectral_norm(self):
        pass  # reference :364-372 matches Conv2d only


class HiFiGANMultiScaleDiscriminator(nn.Module):
    """HiFi-GAN multi-scale discriminator module (discriminator.py:375-447)."""

    def __init__(self, scales=3, downsample_pooling="AvgPool1d",
                 downsample_pooling_params={"kernel_size": 4, "stride": 2, "padding": 2},
                 discriminator_params={"in_channels": 1, "out_channels": 1, "kernel_sizes": [15, 41, 5, 3],
                                       "channels": 128, "max_downsample_channels": 1024, "max_groups": 16,
                                       "bias": True, "downsample_scales": [2, 2, 4, 4, 1],
                                       "nonlinear_activation": "LeakyReLU",
                                       "nonlinear_activation_params": {"negative_slope": 0.1}},
                 follow_official_norm=False):
        super().__init__()
        self.discriminators = nn.ModuleList()
        for i in range(scales):
            params = copy.deepcopy(discriminator_params)
            if follow_official_norm:
                if i == 0:
                    params["use_weight_norm"] = False
                    params["use_spectral_norm"] = True
                else:
                    params["use_weight_norm"] = True
                    params["use_spectral_norm"] = False
            self.discriminators += [HiFiGANScaleDiscriminator(**params)]
        if downsample_pooling != "AvgPool1d":
            raise NotImplementedError(f"{downsample_pooling}: only AvgPool1d is lowered to the HIP path")
        self.pooling = nn.AvgPool1d(**downsample_pooling_params)
        self._pool = (downsample_pooling_params.get("kernel_size"), downsample_pooling_params.get("stride"),
                      downsample_pooling_params.get("padding", 0))

    def _scales(self, x, fn):
        outs = []
        b = x.shape[0]
        k, s, p = self._pool
        s = k if s is None else s
        for f in self.discriminators:
            outs += [fn(f, x)]
            x = DC.AvgPoolFn.apply(x.reshape(b, -1).float(), k, s, p).unsqueeze(1)
        return outs

    def forward(self, x):
        return self._scales(x, lambda f, v: f(v))

    def stash_first_half(self, x):
        with torch.no_grad():
            return self._scales(x, lambda f, v: f.stash_first_half(v))

    def forward_second_half(self, x):
        with torch.no_grad():  # the waveform (a detached prediction) takes no gradient
            pooled = self._scales(x, lambda f, v: v)
        return [f.forward_second_half(v) for f, v in zip(self.discriminators, pooled)]
