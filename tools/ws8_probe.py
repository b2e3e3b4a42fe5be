"""Ablation timing of the eight-wave warp-specialised kernel (conv.hip
k_conv_ws8) against the 12-wave one on the MPD's wide layers at C5 D-step
size (period 2, 32 clips) and the C3 RU128 k7 dgrad.  tune key 13 (ws8
diagnostics): 1 = no DMA in the loop, 2 = no MFMAs, 4 = no loop barriers,
8 = no epilogue.  GPU only; results are garbage in the ablated modes."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "dl-speech-enhancement_amd")]

import torch  # noqa: E402

from sel import _lib as L  # noqa: E402
from sel import convops as CO  # noqa: E402
from sel import dconvops as DC  # noqa: E402
from models.vocoder.modules.discriminator import HiFiGANPeriodDiscriminator  # noqa: E402

dev = torch.device("cuda")
lib = L.lib()


def timed(fn, iters=20):
    for _ in range(3):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    for e0, e1 in ev:
        e0.record()
        fn()
        e1.record()
    torch.cuda.synchronize()
    return sorted(e0.elapsed_time(e1) for e0, e1 in ev)[iters // 2] * 1e3


def modes(tag, fn, flops):
    out = []
    for key37, dbg in ((1, 0), (0, 0), (0, 1), (0, 2), (0, 4), (0, 8), (0, 5), (0, 3)):
        lib.sel_tune(37, key37)
        lib.sel_tune(13, dbg)
        t = timed(fn)
        out.append(f"{'ws12' if key37 else 'ws8'}/dbg{dbg}={t:.1f}us" + (f"({flops / t / 1e6:.0f}TF)" if dbg == 0 else ""))
    lib.sel_tune(37, 0)
    lib.sel_tune(13, 0)
    print(tag, " ".join(out), flush=True)


specs = HiFiGANPeriodDiscriminator(period=2).plan()
period, clips = 2, 32
Lv = (48000 + period - 1) // period
Bs = clips * period
geo = DC.chain_layout(specs, Lv, DC.period_alloc(Lv, specs))
for li in (2, 3, 4):
    sp = specs[li]
    T_in, Ta, T_out, To = geo[li]
    d = DC._fwd_desc(sp, Bs, T_in, Ta, T_out, To, 0.1)
    x = (0.5 * torch.randn(Bs, Ta, sp.cin, device=dev)).to(torch.bfloat16)
    w = torch.randn(sp.cout, sp.cin, sp.Kt, device=dev) / (sp.cin * sp.Kt) ** 0.5
    wp = DC._pack(sp, w, None, torch.bfloat16, 0)
    y = torch.empty(Bs, To, sp.cout, dtype=torch.bfloat16, device=dev)
    b = torch.randn(sp.cout, device=dev)
    flops = 2.0 * Bs * T_out * sp.cout * sp.cin * sp.Kt
    modes(f"MPD p{period} L{li} {sp.cin}->{sp.cout} K{d.K} C{d.S * d.Cg} {DC.kernel(d, torch.bfloat16)[1]}",
          lambda: DC.prim(d, x, wp, y, bias=b), flops)

# C3 RU128 k7 d1 dgrad (T = 2000, 64 clips): aux + res epilogue
d = CO.ConvDesc(64 * 2000, 2000, 128, 128, 7, 1, 6, 0, 1, 0).adjoint()
x = (0.5 * torch.randn(d.rows, d.C, device=dev)).to(torch.bfloat16)
wp = (torch.randn(d.N, d.K, d.C, device=dev) / (d.K * d.C) ** 0.5).to(torch.bfloat16)
a_ = torch.randn(d.rows, d.N, device=dev).to(torch.bfloat16)
r_ = torch.randn(d.rows, d.N, device=dev).to(torch.bfloat16)
lib.sel_tune(4, 1)
modes(f"C3 RU128 k7 dgrad {CO.fwd_kernel_name(d, torch.bfloat16, torch.bfloat16)}",
      lambda: CO.prim(d, x, wp, aux=a_, res=r_), 2.0 * d.rows * d.N * d.C * d.K)
lib.sel_tune(4, 0)
