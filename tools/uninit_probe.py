"""Uninitialised-memory probe for a tests/ddp_product_worker.py case: the same
seeded step run with every torch.empty / empty_like / new_empty poisoned
(filled with NaN, then with a large finite value) against a zero fill; a
result that depends on the fill read memory no kernel wrote.  Per-file blame:
POISON_FILES=a.py,b.py poisons only allocations made from those files.
usage: python tools/uninit_probe.py CASE"""
import os
import sys
import traceback

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "tests"), os.path.join(REPO, "dl-speech-enhancement_amd"), REPO]
import ddp_product_worker as W  # noqa: E402

_empty, _empty_like, _new_empty = torch.empty, torch.empty_like, torch.Tensor.new_empty
FILL = [None]
ONLY = [f for f in os.environ.get("POISON_FILES", "").split(",") if f]


def _caller_ok():
    if not ONLY:
        return True
    st = traceback.extract_stack(limit=4)[-3]
    return any(st.filename.endswith(f) for f in ONLY)


def _poison(t):
    if FILL[0] is not None and t.is_cuda and _caller_ok():
        if t.is_floating_point():
            t.fill_(FILL[0])
        elif t.dtype == torch.uint8:
            t.fill_(255)   # workspaces: every byte 0xFF (a NaN pattern in any float view)
    return t


torch.empty = lambda *a, **k: _poison(_empty(*a, **k))
torch.empty_like = lambda *a, **k: _poison(_empty_like(*a, **k))
torch.Tensor.new_empty = lambda self, *a, **k: _poison(_new_empty(self, *a, **k))


def run(fill):
    FILL[0] = fill
    torch.manual_seed(0)
    r = W.run_case(sys.argv[1], torch.device("cuda"))
    torch.cuda.synchronize()
    FILL[0] = None
    return r


base = run(0.0)
for rep in range(3):   # run-to-run determinism with the same fill
    r = run(0.0)
    diff = [k for k, v in base["grads"].items() if not torch.equal(v, r["grads"][k])]
    print(f"repeat {rep}: {len(diff)} gradients not bit-identical", diff[:6], flush=True)
for fill in (float("nan"), 3.0e4):
    r = run(fill)
    bad = []
    for k, v in base["grads"].items():
        w = r["grads"][k]
        e = ((w.double() - v.double()).norm() / (v.double().norm() + 1e-30)).item()
        if not (e <= 1e-6):
            bad.append((k, e))
    print(f"fill {fill}: {len(bad)} of {len(base['grads'])} gradients differ", bad[:8], flush=True)
