"""Every sel C-ABI call of one eager C3 step, in issue order, with its kernel
tag, event-timed duration and conv descriptor (rows, T, C, N, K, dil, in_elu).

    python tools/call_list.py [B] > gpurun_out/call_list.md

Used to find which layers a kernel instance of the rocprof summary belongs to.
"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "dl-speech-enhancement_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402


class _All:
    def __contains__(self, name):
        return True


def main(B=64):
    import bench
    from sel import _lib as L
    from sel import convops as CO
    dev = torch.device("cuda", 0)
    step = bench.c3_setup(dev, B, 1, 0)
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    descs = []
    orig = L.call

    def call(name, *args, meta=None):
        d = None
        if args and hasattr(args[0], "_obj") and isinstance(args[0]._obj, CO.ConvDesc):
            o = args[0]._obj
            d = (o.rows, o.T, o.C, o.N, o.K, o.dil, o.in_elu)
        descs.append(d)
        return orig(name, *args, meta=meta)

    timer = L.KernelTimer([])
    timer.names = _All()
    L.call = call
    L.TIMER = timer
    try:
        step()
        torch.cuda.synchronize()
    finally:
        L.call = orig
        L.TIMER = None
    print("| # | entry | tag | us | rows, T, C, N, K, dil, in_elu |")
    print("|---|---|---|---|---|")
    tot = 0.0
    for i, ((name, tag, nb, fl, a, b), d) in enumerate(zip(timer.records, descs)):
        us = a.elapsed_time(b) * 1e3
        tot += us
        print(f"| {i} | {name} | `{tag}` | {us:.1f} | {d} |")
    print(f"\n{len(descs)} calls, {tot / 1e3:.3f} ms event-timed")


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 64)
