"""Negative control of tests/test_gpu_ddp.py::test_bucket_waits_for_every_producing_stream:
the same scenario with torch.cuda.Stream.wait_stream disabled inside the
bucket launch (the pre-fix reducer), which should leave the side-stream
gradient unscaled.  usage: python tools/stream_wait_ctrl.py"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "tests"), os.path.join(REPO, "dl-speech-enhancement_amd"), REPO]
import torch.distributed as dist  # noqa: E402
from sel import ddp  # noqa: E402


class _Work:
    def wait(self):
        pass


dist.get_world_size = lambda group=None: 2
dist.all_reduce = lambda t, group=None, async_op=False: _Work()
gpu = torch.device("cuda")
for disable in (False, True):
    orig = ddp.GradBuckets._launch

    def launch(self, bi, _orig=orig):
        if disable:
            w = torch.cuda.Stream.wait_stream
            torch.cuda.Stream.wait_stream = lambda s, o: None
            try:
                return _orig(self, bi)
            finally:
                torch.cuda.Stream.wait_stream = w
        return _orig(self, bi)
    ddp.GradBuckets._launch = launch
    p1 = torch.nn.Parameter(torch.zeros(1 << 20, device=gpu))
    p2 = torch.nn.Parameter(torch.zeros(1 << 10, device=gpu))
    gb = ddp.GradBuckets([p1, p2], bucket_cap_mb=64.0)
    side = torch.cuda.Stream(device=gpu)
    a = torch.randn(2048, 2048, device=gpu)
    torch.cuda.synchronize()
    # y1 built last: its backward (on the side stream) runs first, so the
    # bucket completes with p2, on the current stream
    y2 = (p2 * 5.0).sum()
    with torch.cuda.stream(side):
        y1 = (p1 * 3.0).sum()
    with torch.cuda.stream(side):
        for _ in range(40):
            a = torch.tanh(a @ a * 1e-3)
    (y1 + y2).backward()
    torch.cuda.synchronize()
    print("wait disabled" if disable else "with the wait", "p1.grad values:", p1.grad.unique()[:4].tolist(),
          "p2:", p2.grad.unique().tolist(), flush=True)
    gb.detach()
    ddp.GradBuckets._launch = orig
