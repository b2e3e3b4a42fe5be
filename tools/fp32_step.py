"""The C3 step at fp32 (bench.py's fp32 companion) alone, for kernel profiles:
python tools/fp32_step.py [steps]   (GPU)"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO]

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    dev = torch.device("cuda", 0)
    step = bench.c3_setup(dev, 64, 1, 0, dtype=torch.float32)
    step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    print(f"fp32 C3 step: {(time.perf_counter() - t0) / steps * 1e3:.2f} ms", flush=True)


if __name__ == "__main__":
    main()
