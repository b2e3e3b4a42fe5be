"""A/B of the |X| kernel (sel_stft_mag_fwd, 1024/120/600, B = 2048 x 1 s: the
bench's stft_kernel line) under tune settings, alternating, against the same
run's copy probe.   usage: python tools/stft_ab.py "64=0" "64=1"   (GPU)"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "dl-speech-enhancement_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
from sel import _lib as L  # noqa: E402


def main():
    dev = torch.device("cuda")
    lib = L.lib()
    for rnd in range(3):
        for spec in sys.argv[1:]:
            kv = [tuple(int(v) for v in s.split("=")) for s in spec.split(",") if s]
            prev = [(k, lib.sel_tune(k, v)) for k, v in kv]
            r = bench.stft_kernel_roofline(dev)
            for k, v in prev:
                lib.sel_tune(k, v)
            print(rnd, spec, r["median_launch_us"], "us", r["achieved"], "GB/s", "frac_of_copy_f4", r["frac_of_copy_f4"],
                  flush=True)


if __name__ == "__main__":
    main()
