"""k_pw_bf16 workgroup-count sweep (tune key 43) on the RU256 / RU128 1x1
shapes; usage: python tools/pw_sweep.py [nb ...]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dl-speech-enhancement_amd"))
sys.path.insert(0, os.path.join(REPO, "tools"))

import torch  # noqa: E402

import conv_bench as CB  # noqa: E402
from sel import _lib as L  # noqa: E402


def main():
    nbs = [int(v) for v in sys.argv[1:]] or [0, 128, 256, 384, 512, 768, 1024]
    shapes = [s for s in CB.SHAPES if "1x1" in s[0] and ("256" in s[0] or "128" in s[0])]
    print("| shape | " + " | ".join(f"nb{n}" for n in nbs) + " |")
    for sh in shapes:
        cells = []
        for nb in nbs:
            L.lib().sel_tune(43, nb)
            us, _ = CB.run(sh, 42)
            cells.append(f"{us:.1f}")
        L.lib().sel_tune(43, 0)
        print(f"| {sh[0]} | " + " | ".join(cells) + " |", flush=True)


if __name__ == "__main__":
    main()
