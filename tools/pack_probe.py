"""How many sel_pack_many launches (and jobs each) one C3 step makes.  GPU only."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "dl-speech-enhancement_amd"))
import torch
import bench
from sel import _lib as L
from sel import convops as CO

calls = []
orig = L.call
def spy(name, *args, **kw):
    if name == "sel_pack_many":
        calls.append(args[1])
    return orig(name, *args, **kw)
L.call = spy
CO.L.call = spy
step = bench.c3_setup(torch.device("cuda"), 8, 1, 0)
for i in range(3):
    calls.clear()
    step()
    torch.cuda.synchronize()
    print(f"step {i}: {len(calls)} pack launches, jobs per launch {calls}", flush=True)
