"""Per-shape times of the conv primitive launches (sel_conv_fwd) inside the C3
trainer step: a KernelTimer over the launches, tagged with the descriptor
(rows, T, C, N, K, dil, pad, ELU prologue, aux, res) and the kernel instance.
usage: python tools/layer_times.py [steps]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "dl-speech-enhancement_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
from sel import _lib as L  # noqa: E402
from sel import convops as CO  # noqa: E402

_orig = CO._fwd_meta


def _meta(desc, x, out, wp, aux, res):
    tag, nb, fl = _orig(desc, x, out, wp, aux, res)
    shp = (f"r{desc.rows} T{desc.T} {desc.C}->{desc.N} k{desc.K} d{desc.dil} p{desc.pad} e{desc.in_elu} "
           f"a{int(aux is not None)} r{int(res is not None)}")
    return f"{shp} | {tag}", nb, fl


_call = L.call


def _call_tagged(name, *args, meta=None):
    # the deferred weight-gradient partials (and the fused residual-unit calls) tagged by shape
    if meta is None and name == "sel_conv_wgrad_partials":
        d = args[0]._obj
        tag = (f"wgrad r{d.rows} T{d.T} {d.C}->{d.N} k{d.K} d{d.dil} p{d.pad} e{d.in_elu}")
        meta = (tag, 2 * (d.rows * d.C + d.rows * d.N), 2.0 * d.rows * d.N * d.K * d.C)
    return _call(name, *args, meta=meta)


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    CO._fwd_meta = _meta
    L.call = _call_tagged
    step = bench.c3_setup(torch.device("cuda"), 64, 1, 0)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    L.TIMER = L.KernelTimer(["sel_conv_fwd", "sel_conv_wgrad_partials", "sel_resunit_fwd", "sel_resunit_bwd",
                             "sel_resunit_bwd_wgrad", "sel_wgrad_finish_many"])
    for _ in range(steps):
        step()
    summ = L.TIMER.summary()
    L.TIMER = None
    rows = sorted(summ.items(), key=lambda kv: -kv[1][1])
    tot = 0.0
    for tag, (n, ms, nb, fl) in rows:
        us = ms * 1e3 / n
        tot += ms / steps
        print(f"{ms * 1e3 / steps:8.1f} us/step  n/step {n / steps:4.1f}  avg {us:7.1f} us  "
              f"{nb / n / us / 1e3:6.0f} GB/s  {fl / n / us / 1e6:6.0f} TF/s  {tag}")
    print(f"total {tot:.3f} ms/step")


if __name__ == "__main__":
    main()
