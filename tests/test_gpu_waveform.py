"""GPU parity of the waveform shape loss (losses/waveform_loss.py:15-74) on the
sel_shape_loss kernels: the reference-generated golden (loss 1e-6, gradient
exact up to fp32 summation: 1e-6) and the oracle at C3 size (B=64, 1 s)."""
import numpy as np
import pytest
import torch

from conftest import golden

pytestmark = pytest.mark.gpu


def test_shape_losses_match_reference_golden(gpu):
    from losses import MultiWindowShapeLoss, WaveformShapeLoss
    g = golden("waveform")
    y = torch.from_numpy(g["y"]).to(gpu)
    for tag, mod in (("multi", MultiWindowShapeLoss()), ("w160", WaveformShapeLoss(160))):
        x = torch.from_numpy(g["y_hat"]).to(gpu).requires_grad_(True)
        loss = mod(x, y)
        np.testing.assert_allclose(loss.item(), g[f"{tag}.loss"], rtol=1e-6)
        loss.backward()
        np.testing.assert_allclose(x.grad.cpu().numpy(), g[f"{tag}.grad"], rtol=1e-6, atol=1e-10)


def test_shape_loss_c3_size_vs_oracle(gpu):
    from oracle import ref_ops as R
    from losses import MultiWindowShapeLoss
    gen = torch.Generator().manual_seed(2)
    yh = 0.1 * torch.randn(64, 1, 24000, generator=gen)
    y = 0.1 * torch.randn(64, 1, 24000, generator=gen)
    xr = yh.double().clone().requires_grad_(True)
    lr = R.multi_window_shape_loss(xr, y.double())
    lr.backward()
    xd = yh.to(gpu).requires_grad_(True)
    ld = MultiWindowShapeLoss()(xd, y.to(gpu))
    ld.backward()
    np.testing.assert_allclose(ld.item(), lr.item(), rtol=1e-6)
    e = ((xd.grad.double().cpu() - xr.grad).norm() / xr.grad.norm()).item()
    assert e < 1e-6, e


def test_shape_loss_rejects_target_grad(gpu):
    from losses import WaveformShapeLoss
    a = torch.randn(1, 1, 1000, device=gpu)
    with pytest.raises(RuntimeError, match="y_hat only"):
        WaveformShapeLoss(100)(a, a.clone().requires_grad_(True))
