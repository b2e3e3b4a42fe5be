"""Ablation timings of the sample-tile kernel k_conv_wss (tune key 48 bits:
1 consumers skip the MFMA phase, 2 no DMA, 4 no ELU pass, 8 no output stores)
on the C3 T = 400 shapes, event-timed back-to-back launches.

usage: python tools/wss_probe.py   (GPU)
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dl-speech-enhancement_amd"))
sys.path.insert(0, os.path.join(REPO, "tools"))

import torch  # noqa: E402

import conv_bench as CB  # noqa: E402
from sel import _lib as L  # noqa: E402

MODES = [0, 4, 8, 1, 2, 2 | 4, 1 | 8, 1 | 2 | 4 | 8]


def main():
    lib = L.lib()
    shapes = [s for s in CB.SHAPES if s[2] == 400 and s[5] > 1]
    print("| shape | " + " | ".join(f"dbg{m}" for m in MODES) + " | v27 |")
    print("|---" * (len(MODES) + 2) + "|")
    for sh in shapes:
        cells = []
        for m in MODES:
            lib.sel_tune(48, m)
            us, err = CB.run(sh, 50, iters=30)
            cells.append("-" if us is None else f"{us:.1f}")
        lib.sel_tune(48, 0)
        us27, _ = CB.run(sh, 27, iters=30)
        print(f"| {sh[0]} | " + " | ".join(cells) + f" | {us27:.1f} |", flush=True)
    lib.sel_tune(0, 0)


if __name__ == "__main__":
    main()
