"""The bench's STFT |X| roofline probe on its own (bench.stft_kernel_roofline):
python tools/stft_probe.py [B]  (SEL_LIB=... selects a library build for A/B)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "dl-speech-enhancement_amd")]

import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    r = bench.stft_kernel_roofline(torch.device("cuda"), B)
    print(os.path.basename(os.environ.get("SEL_LIB", "libsel.so")), json.dumps(r), flush=True)
