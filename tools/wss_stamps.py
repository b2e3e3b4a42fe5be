"""Per-block phase stamps of k_conv_wss (tune key 48 bit 4) on the RU256 k7
forward / adjoint shapes: median cycles of [start -> first chunk ready ->
consumer loop done -> tile in LDS -> end] and the in-kernel clock.

usage: python tools/wss_stamps.py [extra dbg bits]   (GPU)
"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dl-speech-enhancement_amd"))

import torch  # noqa: E402

from sel import _lib as L  # noqa: E402
from sel import convops as CO  # noqa: E402


def main():
    extra = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    lib = L.lib()
    dev = torch.device("cuda")
    for name, pad, elu, aux in (("RU256 k7d1 fwd", 6, 1, 0), ("RU256 k7 dgrad", 0, 0, 1)):
        d = CO.ConvDesc(25600, 400, 256, 256, 7, 1, pad, CO.PAD_ZERO, elu, 0)
        x = (0.5 * torch.randn(25600, 256, device=dev)).to(torch.bfloat16)
        wp = (0.05 * torch.randn(256, 7, 256, device=dev)).to(torch.bfloat16)
        a_ = torch.randn(25600, 256, device=dev).to(torch.bfloat16) if aux else None
        out = torch.empty(25600, 256, dtype=torch.bfloat16, device=dev)
        lib.sel_tune(0, 30)
        lib.sel_tune(48, 16 | extra)
        for _ in range(40):  # >= 2 s of back-to-back launches is not needed for ratios; warm the clock a bit
            L.call("sel_conv_fwd", ctypes.byref(d), CO.BF16, CO.BF16, L.ptr(x), L.ptr(wp), None,
                   L.ptr(a_) if aux else None, L.ptr(a_) if aux else None, L.ptr(out), L.stream())
        torch.cuda.synchronize()
        lib.sel_tune(48, 0)
        lib.sel_tune(0, 0)
        st = out.view(-1).view(torch.int64)[: 256 * 16].view(256, 16).cpu().double()
        ws = st[:, 8:16] - st[:, 8:9]
        print("  wave start offsets (median cycles after wave 0):", [int(v) for v in ws.median(0).values.tolist()])
        ph = st[:, 1:5] - st[:, 0:4]
        med = ph.median(0).values
        tot = (st[:, 4] - st[:, 0]).median().item()
        rt = (st[:, 6] - st[:, 5]).median().item()  # 100 MHz ticks
        clk = tot / (rt / 100e6) / 1e9 if rt > 0 else float("nan")
        span = (st[:, 6].max() - st[:, 5].min()).item() / 100.0
        print(f"{name}: cycles start->ready {med[0]:.0f}, loop {med[1]:.0f}, ->tile {med[2]:.0f}, "
              f"epilogue {med[3]:.0f}, total {tot:.0f} ({rt / 100:.1f} us, {clk:.2f} GHz); "
              f"first start -> last end {span:.1f} us", flush=True)


if __name__ == "__main__":
    main()
