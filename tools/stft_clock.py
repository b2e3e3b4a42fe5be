"""Effective shader clock of k_stft_mag_fwd<10> from per-wave s_memtime /
s_memrealtime stamps (a libsel built with -DSEL_STFT_ABL containing bit 8
writes them over the first |X| rows).  usage: SEL_LIB=... python tools/stft_clock.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "dl-speech-enhancement_amd")]

import torch  # noqa: E402

from sel import _lib as L  # noqa: E402

B, T, (n, h, w) = 512, 24000, (1024, 120, 600)
dev = torch.device("cuda")
x = 0.1 * torch.randn(B, T, device=dev)
win = torch.hann_window(w, device=dev)
F, K = 1 + T // h, n // 2 + 1
mag = torch.empty(B, F, K, device=dev)
for _ in range(4):
    L.call("sel_stft_mag_fwd", L.ptr(x), B, T, n, h, w, L.ptr(win), 1e-7, L.ptr(mag), L.stream())
torch.cuda.synchronize()
raw = mag.view(-1)[: 8192 * 16].view(torch.int64).view(-1, 8).cpu()
raw = raw[raw[:, 7] == 0x5354465453544654]
st = raw[:, :4].double()
ok = (st[:, 3] > st[:, 2]) & (st[:, 1] > st[:, 0])
st = st[ok]
raw = raw[ok]
dt, dr = st[:, 1] - st[:, 0], (st[:, 3] - st[:, 2]) / 100e6
span = (st[:, 3].max() - st[:, 2].min()) / 100e6
q = torch.tensor([0.0, 0.1, 0.5, 0.9, 1.0], dtype=torch.float64)
r0 = st[:, 2].min()
start, end = (st[:, 2] - r0) / 100, (st[:, 3] - r0) / 100  # us
print("start us pct", [round(float(v), 1) for v in torch.quantile(start, q)],
      "end us pct", [round(float(v), 1) for v in torch.quantile(end, q)],
      "loop us pct", [round(float(v), 1) for v in torch.quantile(dr * 1e6, q)],
      "late starters", int((start > end.min()).sum()))
print(f"waves {len(st)}  wave loop time median {dr.median() * 1e6:.1f} us  span {span * 1e6:.1f} us  "
      f"clock median {float((dt / dr).median()) / 1e9:.3f} GHz  min {float((dt / dr).min()) / 1e9:.3f} "
      f"max {float((dt / dr).max()) / 1e9:.3f}")

hw, xcc = raw[:, 4], raw[:, 5] & 15
cu = ((hw >> 8) & 15) + 16 * ((hw >> 12) & 1) + 32 * ((hw >> 13) & 7)
loop = dr * 1e6
for x in range(8):
    m = xcc == x
    print(f"xcc {x}: waves {int(m.sum())} loop median {float(loop[m].median()):.1f} us  max {float(loop[m].max()):.1f}")
key = xcc * 1024 + cu
per = {}
for k, t in zip(key.tolist(), loop.tolist()):
    per.setdefault(k, []).append(t)
by_n = {}
for k, ts in per.items():
    by_n.setdefault(len(ts), []).append(sum(ts) / len(ts))
for n_, v in sorted(by_n.items()):
    v.sort()
    print(f"CUs with {n_} waves: {len(v)}  mean loop {sum(v) / len(v):.1f} us  min {v[0]:.1f} max {v[-1]:.1f}")
blk = raw[:, 6]
bl = {}
for b_, t in zip(blk.tolist(), loop.tolist()):
    bl.setdefault(b_, []).append(t)
nw = max(len(v) for v in bl.values())
within = [max(v) - min(v) for v in bl.values() if len(v) == nw]
means = [sum(v) / nw for v in bl.values() if len(v) == nw]
ms = sorted(means)
print("block mean loop pct", [round(ms[int(f * (len(ms) - 1))], 1) for f in (0, 0.05, 0.25, 0.5, 0.75, 0.95, 1)])
print(f"within-block spread median {sorted(within)[len(within) // 2]:.1f} us max {max(within):.1f}; "
      f"block means min {min(means):.1f} median {sorted(means)[len(means) // 2]:.1f} max {max(means):.1f}")
# per CU: blocks ordered by start time, their mean loop times
cub = {}
for k, b_, t, s0 in zip(key.tolist(), blk.tolist(), loop.tolist(), start.tolist()):
    cub.setdefault(k, {}).setdefault(b_, []).append((s0, t))
rank = {}
for k, d in cub.items():
    order = sorted(d.items(), key=lambda kv: min(s for s, _ in kv[1]))
    for r, (b_, v) in enumerate(order):
        rank.setdefault(r, []).append(sum(t for _, t in v) / len(v))
for r, v in sorted(rank.items()):
    print(f"block start rank {r} on its CU: blocks {len(v)} mean loop {sum(v) / len(v):.1f} us")
