"""Diagnostic A/B of the warp-specialised conv kernel (conv.hip k_conv_ws_bf16):
tune key 13 bit 0 = consumers alone, bit 1 = producers alone, bit 2 = no
epilogue; 7 = barriers only (launch floor).  GPU only."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dl-speech-enhancement_amd"))
sys.path.insert(0, os.path.join(REPO, "tools"))

import torch  # noqa: E402

from sel import _lib as L  # noqa: E402
from sel import convops as CO  # noqa: E402
import conv_bench as CB  # noqa: E402


def stamps(name, mode):
    """Per-block realtime stamps (tune key 13 bit 3): start spread, duration and
    blocks per CU of one launch."""
    sh = [s for s in CB.SHAPES if s[0] == name][0]
    _, rows, T, C, N, K, dil, pad, m_, elu, aux, res, bias = sh
    dev = torch.device("cuda")
    d = CO.ConvDesc(rows, T, C, N, K, dil, pad, m_, elu, N if bias else 0)
    x = (0.5 * torch.randn(rows, C, device=dev)).to(torch.bfloat16)
    wp = (0.05 * torch.randn(N, K, C, device=dev)).to(torch.bfloat16)
    lib = L.lib()
    nb = (rows // T) * ((T + 255) // 256) * (N // 128)
    scratch = torch.zeros(nb * 16, device=dev)  # 8 int64 stamps per block (bias_period 0: not a bias)
    lib.sel_tune(0, 27)
    lib.sel_tune(4, 1)
    lib.sel_tune(13, 8 | mode)
    a_ = torch.randn(rows, N, device=dev).to(torch.bfloat16) if aux else None
    r_ = torch.randn(rows, N, device=dev).to(torch.bfloat16) if res else None
    for _ in range(5):
        CO.prim(d, x, wp, bias=scratch, aux=a_, res=r_)
    torch.cuda.synchronize()
    lib.sel_tune(13, 0)
    lib.sel_tune(0, 0)
    lib.sel_tune(4, 0)
    st = scratch.view(torch.int64).view(nb, 8).cpu()
    base = st[:, 0].min()
    s0, s1, s2 = st[:, 0] - base, st[:, 1] - base, st[:, 2] - base
    hw, xcc = st[:, 5], st[:, 6]
    cu = ((hw >> 8) & 15) + 16 * ((hw >> 12) & 1) + 32 * ((hw >> 13) & 7) + 256 * (xcc & 15)
    per = torch.bincount(cu)
    loop = (s1 - s0).double() * 10e-3
    epi = (s2 - s1).double() * 10e-3
    ghz = (st[:, 4] - st[:, 3]).double() / ((st[:, 2] - st[:, 0]).double() * 10.0)
    print(f"{name} mode {mode}: {nb} blocks on {int((per > 0).sum())} CUs (max {int(per.max())}/CU); "
          f"start spread {s0.max().item() * 10e-3:.2f} us; main loop median {loop.median():.2f} "
          f"(max {loop.max():.2f}); epilogue median {epi.median():.2f} (max {epi.max():.2f}); "
          f"first start -> last end {s2.max().item() * 10e-3:.2f} us; clock {ghz.median():.3f} GHz", flush=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "stamps":
        modes = [int(m) for m in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0, 1]
        for m in modes:
            stamps("RU256 k7d1 fwd", m)
            stamps("RU256 k7 dgrad", m)
        return
    names = sys.argv[1].split(",") if len(sys.argv) > 1 else ["RU256 k7d1 fwd"]
    modes = [int(m) for m in (sys.argv[2].split(",") if len(sys.argv) > 2 else "0,1,2,4,3,7".split(","))]
    variants = [int(v) for v in (sys.argv[3].split(",") if len(sys.argv) > 3 else ["27"])]
    lib = L.lib()
    for sh in [s for s in CB.SHAPES if s[0] in names]:
        for v in variants:
            cells = []
            for m in modes:
                lib.sel_tune(13, m)
                us, err = CB.run(sh, v, iters=50)
                cells.append(f"m{m}={us:.1f}" if us else f"m{m}=ERR {err}")
            lib.sel_tune(13, 0)
            print(f"{sh[0]} v{v}: " + "  ".join(cells), flush=True)
    # host-side floor: the same launches through CO.prim with nothing to do on the GPU is not
    # separable; report the python per-call overhead of an empty torch op for scale
    x = torch.empty(1, device="cuda")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(200):
        x.add_(1)
    e1.record()
    torch.cuda.synchronize()
    print(f"empty torch op loop: {e0.elapsed_time(e1) * 1e3 / 200:.1f} us/launch")


if __name__ == "__main__":
    main()
