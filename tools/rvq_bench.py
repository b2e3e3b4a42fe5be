"""Time the RVQ forward kernels at the C3 shape (N = 64*80 rows, 8 x 1024 x 64).
usage: python tools/rvq_bench.py   (GPU)"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "dl-speech-enhancement_amd")]

import torch  # noqa: E402

from sel import _lib as L  # noqa: E402
from sel.vqops import ResidualVQFn  # noqa: E402


def main():
    dev = torch.device("cuda")
    N, D, K, S = (int(v) for v in os.environ.get("RVQ_SHAPE", "5120,64,1024,8").split(","))
    x = torch.randn(N, D, device=dev)
    emb = torch.randn(S, D, K, device=dev)
    lib = L.lib()
    # "v" or "v:g": tune key 2 = v (0 matrix-core, 2 staged, 1 direct), key 39 = g
    # (matrix-core rows per block: 0 = 16, 2 = 2 x 16)
    for vg in os.environ.get("RVQ_VARIANTS", "0,0:2,2,1").split(","):
        v, g = (int(t) for t in (vg.split(":") + ["0"])[:2])
        lib.sel_tune(2, v)
        lib.sel_tune(39, g)
        for _ in range(3):
            ResidualVQFn.apply(x, emb, 1.0)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            ResidualVQFn.apply(x, emb, 1.0)
        e1.record()
        torch.cuda.synchronize()
        print(f"{(N, D, K, S)} variant {vg}: {e0.elapsed_time(e1) / 20 * 1e3:.1f} us per RVQ forward (+finish)",
              flush=True)
    lib.sel_tune(2, 0)
    lib.sel_tune(39, 0)


if __name__ == "__main__":
    main()
