"""Which torch ops launch GPU kernels inside the C3 trainer step (the glue
around the sel kernels): torch.profiler over 2 steps, aten ops with device
time, grouped by a short Python stack.  usage: python tools/glue_probe.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "dl-speech-enhancement_amd")]

import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

import bench  # noqa: E402


def main():
    step = bench.c3_setup(torch.device("cuda"), 64, 1, 0)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        for _ in range(2):
            step()
        torch.cuda.synchronize()
    ka = prof.key_averages(group_by_stack_n=6)
    rows = [e for e in ka if e.key.startswith("aten::") and e.device_time_total > 0]
    rows.sort(key=lambda e: -e.device_time_total)
    for e in rows[:30]:
        stack = [s for s in e.stack if "site-packages" not in s and "dist-packages" not in s][:4]
        print(f"{e.device_time_total / 2:8.1f} us/step  n={e.count // 2:3d}  {e.key:28s} | " + " <- ".join(stack))


if __name__ == "__main__":
    main()
