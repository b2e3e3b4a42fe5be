"""Timing probe of one discriminator layer's forward and weight gradient on the
dconv primitive (the MSD first conv by default: 1 -> 128 channels, k15, pad 7,
B = 32 x 48000).  usage: python tools/dconv_probe.py [cin cout Kt stride pad groups B T]"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "dl-speech-enhancement_amd")]

import torch  # noqa: E402

from sel import _lib as L  # noqa: E402
from sel import dconvops as D  # noqa: E402

a = [int(v) for v in sys.argv[1:9]] if len(sys.argv) > 8 else [1, 128, 15, 1, 7, 1, 32, 48000]
cin, cout, Kt, stride, pad, groups, B, T = a
dev = torch.device("cuda")
lib = L.lib()
sp = D.LayerSpec(cin, cout, Kt, stride, pad, groups, True)
To = sp.t_out(T)
Ta = (T + stride - 1) // stride * stride
x = (0.1 * torch.randn(B, Ta, cin, device=dev)).to(torch.bfloat16)
desc = D._fwd_desc(sp, B, T, Ta, To, To, 0.1)
w = 0.1 * torch.randn(cout, cin // groups, Kt, device=dev)
wp = D._pack(sp, w, None, torch.bfloat16, 0)
out = torch.empty(B, To, cout, device=dev, dtype=torch.bfloat16)
g = (0.1 * torch.randn(B, To, cout, device=dev)).to(torch.bfloat16)
gw = torch.empty(cout, cin // groups, Kt, device=dev)
gb = torch.empty(cout, device=dev)


def fwd():
    L.call("sel_dconv_fwd", ctypes.byref(desc), 1, L.ptr(x), L.ptr(wp), None, None, None, L.ptr(out), L.stream())


def wg():
    ws = L.workspace(lib.sel_dconv_wgrad_workspace(ctypes.byref(desc), 1), dev)
    L.call("sel_dconv_wgrad", ctypes.byref(desc), 1, L.ptr(g), L.ptr(x), cout, cin // groups, Kt, stride, pad, None,
           None, L.ptr(gw), None, L.ptr(gb), L.ptr(ws), ws.numel(), L.stream())


def timed(fn, iters=10):
    for _ in range(2):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    for e0, e1 in ev:
        e0.record()
        fn()
        e1.record()
    torch.cuda.synchronize()
    return sum(e0.elapsed_time(e1) for e0, e1 in ev) / iters * 1e3


if os.environ.get("PF_AB"):  # forward tile A/B of the register-prefetched MFMA kernel (tune key 19)
    lib.sel_tune(19, 0)
    fwd()
    ref = out.clone()
    for v in (0, 1, 2, 3, 0):
        lib.sel_tune(19, v)
        fwd()
        torch.cuda.synchronize()
        print(f"layer {a} pf tile variant {v}: fwd {timed(fwd):.1f} us  same as default: {bool(torch.equal(out, ref))}",
              flush=True)
    lib.sel_tune(19, 0)
    sys.exit(0)
lib.sel_tune(18, 1)
fwd()
ref = out.clone()
lib.sel_tune(18, 0)
fwd()
torch.cuda.synchronize()
print("staged vs unstaged short forward: max |diff|", float((out.float() - ref.float()).abs().max()),
      "bit-identical", bool(torch.equal(out, ref)), "| unstaged", f"{(lib.sel_tune(18, 1), timed(fwd))[1]:.1f} us",
      flush=True)
lib.sel_tune(18, 1)
wg()
gw_ref, gb_ref = gw.clone(), gb.clone()
t_old = timed(wg)
lib.sel_tune(18, 0)
wg()
torch.cuda.synchronize()
rel = float((gw - gw_ref).norm() / gw_ref.norm()), float((gb - gb_ref).norm() / gb_ref.norm())
print(f"staged vs unstaged short wgrad: rel diff w {rel[0]:.2e} b {rel[1]:.2e} | unstaged {t_old:.1f} us", flush=True)
for knob in (0, 1):
    lib.sel_tune(9, knob)
    print(f"layer {a} tune9={knob}: fwd {timed(fwd):.1f} us  wgrad {timed(wg):.1f} us  "
          f"path={lib.sel_dconv_kernel(ctypes.byref(desc), 1, None, 0)}", flush=True)
lib.sel_tune(9, 0)
