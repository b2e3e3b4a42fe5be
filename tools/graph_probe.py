"""Eager vs HIP-graph replay of the C3 denoise-trainer step (1 GPU).
usage: python tools/graph_probe.py [steps]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "dl-speech-enhancement_amd")]

import torch  # noqa: E402

import bench  # noqa: E402


def timed(fn, steps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda")
    step = bench.c3_setup(dev, 64, 1, 0, graph=True)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            step()
    torch.cuda.current_stream().wait_stream(s)
    print(f"eager: {timed(step, steps):.3f} ms/step", flush=True)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step()
    print("captured", flush=True)
    g.replay()
    torch.cuda.synchronize()
    print(f"graph: {timed(g.replay, steps):.3f} ms/step", flush=True)
    print(f"eager: {timed(step, steps):.3f} ms/step", flush=True)


if __name__ == "__main__":
    main()
