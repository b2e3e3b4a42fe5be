"""Microbenchmark of the conv primitive on the C3 layer shapes (bf16), A/B over
kernel variants inside ONE process (sel_tune key 0).

usage: python tools/conv_bench.py [variants...]    (GPU)
"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dl-speech-enhancement_amd"))

import torch  # noqa: E402

from sel import _lib as L  # noqa: E402
from sel import convops as CO  # noqa: E402

Z, R = CO.PAD_ZERO, CO.PAD_REPLICATE
# name, rows, T, C, N, K, dil, pad, mode, in_elu, aux, res, bias
SHAPES = [
    ("first 1->32 k7", 1536000, 24000, 1, 32, 7, 1, 6, Z, 0, 0, 0, 0),
    ("last dgrad 1->32 k7", 1536000, 24000, 1, 32, 7, 1, 0, Z, 0, 0, 0, 0),
    ("last 32->1 k7", 1536000, 24000, 32, 1, 7, 1, 6, Z, 0, 0, 0, 1),
    ("RU32 k7d9 fwd", 1536000, 24000, 32, 32, 7, 9, 54, Z, 1, 0, 0, 0),
    ("RU32 1x1 fwd", 1536000, 24000, 32, 32, 1, 1, 0, Z, 1, 0, 1, 0),
    ("RU32 k7d9 dgrad", 1536000, 24000, 32, 32, 7, 9, 0, Z, 0, 1, 1, 0),
    ("RU32 1x1 dgrad", 1536000, 24000, 32, 32, 1, 1, 0, Z, 0, 1, 0, 0),
    ("down0 96->64 k3", 512000, 8000, 96, 64, 3, 1, 2, Z, 0, 0, 0, 1),
    ("RU64 k7d3 fwd", 512000, 8000, 64, 64, 7, 3, 18, Z, 1, 0, 0, 0),
    ("RU64 1x1 fwd", 512000, 8000, 64, 64, 1, 1, 0, Z, 1, 0, 1, 0),
    ("RU64 k7d3 dgrad", 512000, 8000, 64, 64, 7, 3, 0, Z, 0, 1, 1, 0),
    ("RU64 1x1 dgrad", 512000, 8000, 64, 64, 1, 1, 0, Z, 0, 1, 0, 0),
    ("up3 dgrad 96->64 k2", 512000, 8000, 96, 64, 2, 1, 0, Z, 0, 0, 0, 0),
    ("up3 64->96 k2 rep", 512000, 8000, 64, 96, 2, 1, 1, R, 0, 0, 0, 1),
    ("down0 dgrad 64->96 k3", 512000, 8000, 64, 96, 3, 1, 0, Z, 0, 0, 0, 0),
    ("RU128 k7d9 fwd", 128000, 2000, 128, 128, 7, 9, 54, Z, 1, 0, 0, 0),
    ("RU128 k7d9 dgrad", 128000, 2000, 128, 128, 7, 9, 0, Z, 0, 1, 1, 0),
    ("RU128 1x1 fwd", 128000, 2000, 128, 128, 1, 1, 0, Z, 1, 0, 1, 0),
    ("RU256 1x1 fwd", 25600, 400, 256, 256, 1, 1, 0, Z, 1, 0, 1, 0),
    ("RU256 1x1 dgrad", 25600, 400, 256, 256, 1, 1, 0, Z, 0, 1, 0, 0),
    ("down1 256->128 k3", 128000, 2000, 256, 128, 3, 1, 2, Z, 0, 0, 0, 1),
    ("up k2 128->256 rep", 128000, 2000, 128, 256, 2, 1, 1, R, 0, 0, 0, 1),
    ("up k2 dgrad 256->128", 128000, 2000, 256, 128, 2, 1, 0, Z, 0, 0, 0, 0),
    ("up k2 256->640 rep", 25600, 400, 256, 640, 2, 1, 1, R, 0, 0, 0, 1),
    ("up k2 dgrad 640->256", 25600, 400, 640, 256, 2, 1, 0, Z, 0, 0, 0, 0),
    ("RU256 k7d1 fwd", 25600, 400, 256, 256, 7, 1, 6, Z, 1, 0, 0, 0),
    ("RU256 k7 dgrad", 25600, 400, 256, 256, 7, 1, 0, Z, 0, 1, 1, 0),
    ("down2 640->256 k3", 25600, 400, 640, 256, 3, 1, 2, Z, 0, 0, 0, 1),
    ("down3 1280->512 k3", 5120, 80, 1280, 512, 3, 1, 2, Z, 0, 0, 0, 1),
    ("dec conv1 64->512", 5120, 80, 64, 512, 7, 1, 6, Z, 0, 0, 0, 0),
    ("up0 512->1280 k2", 5120, 80, 512, 1280, 2, 1, 1, R, 0, 0, 0, 1),
    ("up0 dgrad 1280->512 k2", 5120, 80, 1280, 512, 2, 1, 0, Z, 0, 0, 0, 0),
    ("down3 dgrad 512->1280 k3", 5120, 80, 512, 1280, 3, 1, 0, Z, 0, 0, 0, 0),
    ("dec conv1 dgrad 512->64 k7", 5120, 80, 512, 64, 7, 1, 0, Z, 0, 0, 0, 0),
]


def run(shape, variant, iters=20):
    name, rows, T, C, N, K, dil, pad, mode, elu, aux, res, bias = shape
    dev = torch.device("cuda")
    d = CO.ConvDesc(rows, T, C, N, K, dil, pad, mode, elu, N if bias else 0)
    x = (0.5 * torch.randn(rows, C, device=dev)).to(torch.bfloat16)
    wp = (0.05 * torch.randn(N, K, C, device=dev)).to(torch.bfloat16)
    b = torch.randn(N, device=dev) if bias else None
    a_ = torch.randn(rows, N, device=dev).to(torch.bfloat16) if aux else None
    r_ = torch.randn(rows, N, device=dev).to(torch.bfloat16) if res else None
    # variants 30-33 = the weight-stationary thin kernel (tune key 4 = 0):
    # 30 default, 31 one tile per workgroup (key 5), 32 alternative tile rows
    # (key 6), 33 both; any other variant runs with the thin kernel off so the
    # tiled variants stay comparable
    # 34/35: default rows with the epilogue prefetch (+ split loop) on / off for
    # every instance with epilogue operands (key 12 flips kThinEpfDefault =
    # 0b101, key 11 bit 0 = off); 36/37: the same with key 6 flipping every
    # instance's tile rows (kThinEpfAlt instances flip back under 34/36)
    # 41 / 42: the defaults with the pointwise kernel off / also at 128 channels (tune key 42)
    thin = 30 <= variant <= 37 or variant in (41, 42)
    L.lib().sel_tune(42, {41: 1, 42: 2}.get(variant, 0))
    L.lib().sel_tune(4, 0 if thin else 1)
    L.lib().sel_tune(5, 1 << 30 if variant in (31, 33) else 0)
    L.lib().sel_tune(6, 127 if variant in (32, 33, 36, 37) else 0)
    L.lib().sel_tune(12, 127 ^ 0b101 if variant in (34, 36) else 0)
    L.lib().sel_tune(11, 1 if variant in (35, 37) else 0)
    # 50: the sample-tile kernel k_conv_wss (tune key 0 = 30)
    L.lib().sel_tune(0, 0 if thin or variant == 0 else (30 if variant == 50 else variant))
    try:
        for _ in range(3):
            y = CO.prim(d, x, wp, bias=b, aux=a_, res=r_)
    except L.SelError as e:
        return None, str(e)[:40]
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        y = CO.prim(d, x, wp, bias=b, aux=a_, res=r_)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / iters
    del y
    return us, None


def main():
    variants = [int(v) for v in sys.argv[1:]] or [30, 0, 21, 22, 23, 24]
    L.lib()
    print("| shape | " + " | ".join(f"v{v}" for v in variants) + " | best | GB/s | TF/s |")
    print("|---" * (len(variants) + 4) + "|")
    for sh in [x for x in SHAPES if os.environ.get("SHAPE", "") in x[0]]:
        name, rows, T, C, N, K, dil, pad, mode, elu, aux, res, bias = sh
        times = []
        for v in variants:
            us, err = run(sh, v)
            times.append(us)
        ok = [(t, v) for t, v in zip(times, variants) if t is not None]
        best_t, best_v = min(ok)
        nbytes = 2 * (rows * C + rows * N * (1 + aux + res) + N * K * C)
        flops = 2.0 * rows * N * K * C
        cells = " | ".join("-" if t is None else f"{t:.1f}" for t in times)
        print(f"| {name} | {cells} | v{best_v} | {nbytes / best_t / 1e3:.0f} | {flops / best_t / 1e6:.0f} |",
              flush=True)
    for key in (0, 4, 5, 6, 7, 11, 12, 42):
        L.lib().sel_tune(key, 0)


if __name__ == "__main__" and os.environ.get("WGRAD", "0") != "1":
    main()


WG_SHAPES = [s for s in SHAPES if "dgrad" not in s[0] and os.environ.get("SHAPE", "") in s[0]]


def run_wgrad(shape, variant, iters=10):
    name, rows, T, C, N, K, dil, pad, mode, elu, aux, res, bias = shape
    dev = torch.device("cuda")
    d = CO.ConvDesc(rows, T, C, N, K, dil, pad, mode, elu, N if bias else 0)
    x = (0.5 * torch.randn(rows, C, device=dev)).to(torch.bfloat16)
    g = (0.5 * torch.randn(rows, N, device=dev)).to(torch.bfloat16)
    L.lib().sel_tune(1, variant)
    try:
        for _ in range(2):
            CO.wgrad(d, g, x, bool(bias))
    except L.SelError as e:
        return None
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        CO.wgrad(d, g, x, bool(bias))
    e1.record()
    torch.cuda.synchronize()
    L.lib().sel_tune(1, 0)
    return e0.elapsed_time(e1) * 1e3 / iters


def main_wgrad():
    targets = [int(t) for t in os.environ.get("WG_TARGETS", "").split(",") if t]
    if targets:  # sweep the workgroup-count target (tune key 10) of the default path
        print("\n| wgrad shape | " + " | ".join(f"t{t}" for t in targets) + " |")
        print("|---" * (len(targets) + 1) + "|")
        for sh in WG_SHAPES:
            cells = []
            for t in targets:
                L.lib().sel_tune(10, t)
                us = run_wgrad(sh, 0)
                cells.append("-" if us is None else f"{us:.1f}")
            L.lib().sel_tune(10, 0)
            print(f"| {sh[0]} | " + " | ".join(cells) + " |", flush=True)
        return
    print("\n| wgrad shape | fast (us) | generic (us) | GB/s | TF/s |\n|---|---|---|---|---|")
    for sh in WG_SHAPES:
        name, rows, T, C, N, K, dil, pad, mode, elu, aux, res, bias = sh
        t0, t1 = run_wgrad(sh, int(os.environ.get("WG_A", "0"))), run_wgrad(sh, int(os.environ.get("WG_B", "1")))
        nbytes = 2 * (rows * C + rows * N)
        flops = 2.0 * rows * N * K * C
        print(f"| {name} | {t0:.1f} | {t1:.1f} | {nbytes / t0 / 1e3:.0f} | {flops / t0 / 1e6:.0f} |", flush=True)


if __name__ == "__main__" and os.environ.get("WGRAD", "0") == "1":
    main_wgrad()
