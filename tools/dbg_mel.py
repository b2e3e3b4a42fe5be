"""Locate log-mel backward mismatches against the fp64 oracle (GPU debug aid)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "dl-speech-enhancement_amd")]

import torch  # noqa: E402

from oracle import ref_ops as R  # noqa: E402
from losses import MelSpectrogram  # noqa: E402

for n, h, wl in [(1024, 256, 1024), (2048, 300, 2048), (1024, 120, 600), (2048, 240, 1200), (512, 50, 240)]:
    m = MelSpectrogram(fs=24000, fft_size=n, hop_size=h, win_length=wl, num_mels=80, fmin=0, fmax=12000,
                       log_base=None)
    g = torch.Generator().manual_seed(11)
    x = 0.1 * torch.randn(2, 24000, generator=g)
    F = 1 + 24000 // h
    up = torch.randn(2, 80, F, generator=g)
    xr = x.double().clone().requires_grad_(True)
    o = R.melspec(xr, n, h, wl, m.window.double(), m.melmat.double(), 1e-10, None)
    o.backward(up.double())
    md = m.cuda()
    xd = x.cuda().requires_grad_(True)
    od = md(xd)
    od.backward(up.cuda())
    fe = ((od.double().cpu() - o.detach()).norm() / o.detach().norm()).item()
    gd = xd.grad.double().cpu()
    e = (gd - xr.grad).abs()
    print(n, "fwd rel", fe, "grad rel", (e.norm() / xr.grad.norm()).item(), "nan ours", int(gd.isnan().sum()), "nan ref", int(xr.grad.isnan().sum()))
    big = (e > 1e-2 * xr.grad.abs().max()).nonzero()
    print("  bad samples", big.shape[0], "first", big[:10, 1].tolist(), "last", big[-10:, 1].tolist())
    blocks = (e[0].reshape(-1, 1000).norm(dim=1) / xr.grad[0].reshape(-1, 1000).norm(dim=1))
    print("  per-1000-sample rel err", [round(v, 4) for v in blocks.tolist()])

# the golden L1 path (tests/test_gpu_spectral.py::test_mel_matches_reference_golden)
import numpy as np  # noqa: E402
from losses import MultiMelSpectrogramLoss  # noqa: E402
gz = np.load(os.path.join(REPO, "tests", "golden", "mel.npz"))
p24 = dict(fs=24000, fft_sizes=[2048], hop_sizes=[300], win_lengths=[None], window="hann_window",
           num_mels=80, fmin=0, fmax=24000, log_base=None)
ml = MultiMelSpectrogramLoss(**p24)
mt = ml.mel_transfers[0]
yh, y = torch.from_numpy(gz["y_hat"]), torch.from_numpy(gz["y"])
print("golden shapes", tuple(yh.shape), tuple(y.shape))
yr = yh.double().clone().requires_grad_(True)
lr = R.multi_mel_loss(yr, y.double(), [(2048, 300, 2048)], [mt.window.double()], [mt.melmat.double()], 1e-10, None)
lr.backward()
mld = ml.cuda()
yd = yh.cuda().requires_grad_(True)
ld = mld(yd, y.cuda())
ld.backward()
gd = yd.grad.double().cpu().reshape(yr.grad.shape)
e = (gd - yr.grad).abs()
print("loss", ld.item(), lr.item(), "grad rel", (e.norm() / yr.grad.norm()).item(), "nan", int(gd.isnan().sum()))
flat_e, flat_r = e.reshape(e.shape[0], -1), yr.grad.reshape(e.shape[0], -1)
for b in range(flat_e.shape[0]):
    blocks = flat_e[b].reshape(-1, 1000).norm(dim=1) / flat_r[b].reshape(-1, 1000).norm(dim=1)
    print("  b", b, [round(v, 4) for v in blocks.tolist()])

# default-parameter multi-resolution loss (the test's meldef part), per resolution
mdef = MultiMelSpectrogramLoss()
for i, mt in enumerate(mdef.mel_transfers):
    print("res", i, mt.fft_size if hasattr(mt, "fft_size") else "", getattr(mt, "hop_size", ""),
          tuple(mt.window.shape), tuple(mt.melmat.shape), getattr(mt, "log_base", ""))
mdd = mdef.cuda()
yd = yh.cuda().requires_grad_(True)
ld = mdd(yd, y.cuda())
ld.backward()
print("meldef loss", ld.item(), "golden", float(gz["meldef.loss"]))
gref = torch.from_numpy(gz["meldef.grad"]).double()
gd = yd.grad.double().cpu().reshape(gref.shape)
print("meldef grad rel vs golden fp32", ((gd - gref).norm() / gref.norm()).item())

# per default resolution, L1 path, vs the fp64 oracle
for (n, h, wl) in [(1024, 120, 600), (2048, 240, 1200), (512, 50, 240)]:
    one = MultiMelSpectrogramLoss(fft_sizes=[n], hop_sizes=[h], win_lengths=[wl])
    mt = one.mel_transfers[0]
    yr = yh.double().clone().requires_grad_(True)
    lr = R.multi_mel_loss(yr, y.double(), [(n, h, wl)], [mt.window.double()], [mt.melmat.double()], 1e-10, 10.0)
    lr.backward()
    yd = yh.cuda().requires_grad_(True)
    ld = one.cuda()(yd, y.cuda())
    ld.backward()
    gd = yd.grad.double().cpu().reshape(yr.grad.shape)
    e = (gd - yr.grad)
    print(n, "L1 loss", ld.item(), lr.item(), "grad rel", (e.norm() / yr.grad.norm()).item())
    fe = e.reshape(2, -1)
    fr_ = yr.grad.reshape(2, -1)
    for b in range(2):
        print("   b", b, [round(v, 3) for v in (fe[b].reshape(-1, 2000).norm(dim=1) / fr_[b].reshape(-1, 2000).norm(dim=1)).tolist()])

# near-ties of the L1 sign at the start of signal 1 (1024/120/600)
one = MultiMelSpectrogramLoss(fft_sizes=[1024], hop_sizes=[120], win_lengths=[600])
mt = one.mel_transfers[0]
m64h = R.melspec(yh.double(), 1024, 120, 600, mt.window.double(), mt.melmat.double(), 1e-10, 10.0)
m64y = R.melspec(y.double(), 1024, 120, 600, mt.window.double(), mt.melmat.double(), 1e-10, 10.0)
mtd = mt.cuda()
m32h = mtd(yh.cuda()).double().cpu()
m32y = mtd(y.cuda()).double().cpu()
d64 = (m64h - m64y)[1, :, :12]
d32 = (m32h - m32y)[1, :, :12]
flip = torch.sign(d64) != torch.sign(d32)
print("sign flips (b=1, frames<12):", int(flip.sum()), "min |d64| at flips", d64[flip].abs().min().item() if flip.any() else None,
      "max |d64| at flips", d64[flip].abs().max().item() if flip.any() else None)
print("yh vs y first samples b=1 max|diff|", (yh[1, 0, :3000] - y[1, 0, :3000]).abs().max().item(),
      "max|y|", y[1, 0, :3000].abs().max().item())
