"""Run-to-run determinism of a tests/ddp_product_worker.py case under
allocator churn (random-size tensors allocated, written and freed on the
current stream between and around runs): a cross-stream memory race shows as
gradients that differ from the first run.  usage: python tools/race_probe.py CASE N"""
import os
import random
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "tests"), os.path.join(REPO, "dl-speech-enhancement_amd"), REPO]
import ddp_product_worker as W  # noqa: E402

dev = torch.device("cuda")
rng = random.Random(1)


def churn():
    keep = [torch.full((rng.randint(1, 1 << 22),), float("nan"), device=dev) for _ in range(rng.randint(2, 12))]
    for t in keep:
        t.mul_(2.0)
    del keep


def run():
    churn()
    torch.manual_seed(0)
    r = W.run_case(sys.argv[1], dev)
    churn()
    torch.cuda.synchronize()
    return r["grads"]


base = run()
n = int(sys.argv[2])
bad = 0
for i in range(n):
    g = run()
    diff = [k for k, v in base.items() if not torch.equal(v, g[k])]
    if diff:
        bad += 1
        e = max(((g[k].double() - base[k].double()).norm() / (base[k].double().norm() + 1e-30)).item() for k in diff)
        print(f"run {i}: {len(diff)} gradients differ, max rel {e:.3g}", diff[:4], flush=True)
print(f"{bad} of {n} runs differed (SEL_D_STREAMS={os.environ.get('SEL_D_STREAMS', '8')})", flush=True)
