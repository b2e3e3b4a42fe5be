"""Host issue time vs GPU time of the C3 denoise-trainer step (1 GPU): the
per-step wall time of step() without a sync (the Python / launch issue cost)
against the synchronised per-step time, plus a cProfile of the host side.
usage: python tools/host_probe.py [steps]"""
import cProfile
import io
import os
import pstats
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "dl-speech-enhancement_amd")]

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda")
    step = bench.c3_setup(dev, 64, 1, 0)
    for _ in range(5):
        step()
    torch.cuda.synchronize()
    host = []
    t0 = time.perf_counter()
    for _ in range(steps):
        h0 = time.perf_counter()
        step()
        host.append(time.perf_counter() - h0)
    torch.cuda.synchronize()
    tot = (time.perf_counter() - t0) / steps
    host.sort()
    print(f"synchronised {tot * 1e3:.3f} ms/step; host issue per step median {host[len(host) // 2] * 1e3:.3f} ms "
          f"(min {host[0] * 1e3:.3f}, max {host[-1] * 1e3:.3f})", flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
    print(s.getvalue()[:6000])


if __name__ == "__main__":
    main()
