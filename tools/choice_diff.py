"""Which kernel choices differ between the C3 step at two per-GPU batch sizes?

    python tools/choice_diff.py 8 16

Runs bench.c3_setup's step once per batch size with every sel C-ABI call
recorded (entry name, kernel tag from the call's timer meta, and the integer
arguments), then prints the calls whose tag or integer arguments other than
the row-count-derived ones differ.  Used to pin the data-parallel GPU test
(tests/test_gpu_ddp.py "bench": 8 clips per rank against 16 in one process).
"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "dl-speech-enhancement_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402


def record(B):
    import bench
    from sel import _lib as L
    dev = torch.device("cuda", 0)
    step = bench.c3_setup(dev, B, 1, 0)
    step()
    torch.cuda.synchronize()
    log = []
    orig = L.call

    def call(name, *args, meta=None):
        tag = None
        if meta is not None:
            m = meta() if callable(meta) else meta
            tag = m[0] if m else None
        ints = [a for a in args if isinstance(a, int)]
        desc = None
        if args and isinstance(args[0], ctypes._Pointer if hasattr(ctypes, "_Pointer") else object):
            pass
        try:
            d = args[0]._obj if hasattr(args[0], "_obj") else None
            if d is not None and hasattr(d, "_fields_"):
                desc = {f[0]: getattr(d, f[0]) for f in d._fields_ if f[0] not in ("rows",)}
        except Exception:
            pass
        log.append((name, tag, ints, desc))
        return orig(name, *args, meta=meta)
    L.call = call
    try:
        step()
        torch.cuda.synchronize()
    finally:
        L.call = orig
    return log


def main():
    b1, b2 = int(sys.argv[1]), int(sys.argv[2])
    l1, l2 = record(b1), record(b2)
    print(f"calls: B={b1}: {len(l1)}, B={b2}: {len(l2)}")
    n = 0
    for i, (a, b) in enumerate(zip(l1, l2)):
        if a[0] != b[0] or a[1] != b[1] or a[3] != b[3]:
            n += 1
            print(i, a[0], "|", a[1], "|", b[1], "|", a[3] if a[3] != b[3] else "")
        elif a[2] != b[2]:
            print(i, a[0], "ints", a[2], b[2])
    print("differing tags/descs:", n)


if __name__ == "__main__":
    main()
