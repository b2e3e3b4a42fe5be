"""Fused 32-channel residual unit (k_ru32_fwd / k_ru32_bwd) vs the primitive
calls it replaces, at the C3 size (B = 64 x 24000), per dilation.  GPU only."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dl-speech-enhancement_amd"))
import torch
from sel import convops as CO

def timed(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters

gpu = torch.device("cuda")
# RU_C=64: the 64-channel units at their C3 length (T = 8000)
C = int(os.environ.get("RU_C", "32"))
B, T = 64, (24000 if C == 32 else 8000)
x = (0.5 * torch.randn(B * T, C, device=gpu)).to(torch.bfloat16)
h = (0.5 * torch.randn(B * T, C, device=gpu)).to(torch.bfloat16)
g = (0.5 * torch.randn(B * T, C, device=gpu)).to(torch.bfloat16)
w1 = 0.1 * torch.randn(C, C, 7, device=gpu)
w2 = 0.2 * torch.randn(C, C, 1, device=gpu)
b1 = torch.randn(C, device=gpu)
b2 = torch.randn(C, device=gpu)
MB = B * T * C * 2 / 1e6
from sel import _lib as L
if len(sys.argv) > 1:  # diagnostic store-skip modes of the fused forward (tune key 15)
    d1 = CO.ConvDesc(B * T, T, C, C, 7, 9, 54, CO.PAD_ZERO, 1, C)
    wp1, wd1 = CO.PACKS.get(CO.PACK_FWD, w1, 1, torch.bfloat16)
    wp2, wd2 = CO.PACKS.get(CO.PACK_FWD, w2, 1, torch.bfloat16)
    for m in (0, 1, 2, 3):
        L.lib().sel_tune(15, m)
        print(f"fwd dil 9 mode {m}: {timed(lambda: CO.resunit_fwd(d1, x, wp1, b1, wp2, b2)):.1f} us", flush=True)
    L.lib().sel_tune(15, 0)
for dil in (1, 3, 9):
    d1 = CO.ConvDesc(B * T, T, C, C, 7, dil, 6 * dil, CO.PAD_ZERO, 1, C)
    d2 = CO.ConvDesc(B * T, T, C, C, 1, 1, 0, CO.PAD_ZERO, 1, C)
    wp1, wd1 = CO.PACKS.get(CO.PACK_FWD, w1, 1, torch.bfloat16)
    wp2, wd2 = CO.PACKS.get(CO.PACK_FWD, w2, 1, torch.bfloat16)
    f = timed(lambda: CO.resunit_fwd(d1, x, wp1, b1, wp2, b2))
    f2 = timed(lambda: CO.prim(d2, CO.prim(d1, x, wp1, bias=b1), wp2, bias=b2, res=x))
    bw = timed(lambda: CO.resunit_bwd(d1, g, h, x, wd1, wd2, True))
    bw0 = timed(lambda: CO.resunit_bwd(d1, g, h, x, wd1, wd2, False))
    b2c = timed(lambda: CO.prim(d1.adjoint(), CO.prim(d2.adjoint(), g, wd2, aux=h), wd1, aux=x, res=g))
    # gx + both weight gradients (k_ru32_bwdw / k_ru64_bwdw), with the finish reduction
    bww = timed(lambda: CO.resunit_bwd_wgrad(d1, g, h, x, wd1, wd2, (C, C, 7), (C, C, 1), True, True, None, None))
    print(f"dil {dil}: fwd fused {f:.1f} us ({3 * MB / f:.2f} TB/s) vs two calls {f2:.1f}; "
          f"bwd fused {bw:.1f} ({5 * MB / bw:.2f} TB/s) / no-gh {bw0:.1f} ({4 * MB / bw0:.2f} TB/s) vs two calls {b2c:.1f}; "
          f"bwd+wgrad {bww:.1f} ({4 * MB / bww:.2f} TB/s incl. finish)",
          flush=True)
