"""Stream-copy probe (sel_probe_copy_f4) variants on 1 GiB buffers: the HBM
denominator bench.py's stft_kernel line uses.  usage: python tools/copy_probe.py (GPU)"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dl-speech-enhancement_amd"))

import torch  # noqa: E402

from sel import _lib as L  # noqa: E402


def main():
    dev = torch.device("cuda")
    src = torch.randn(2 ** 28, device=dev)
    dst = torch.empty_like(src)
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    nbytes = 2 * src.numel() * 4

    def timed(fn, iters=10):
        for _ in range(3):
            fn()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
        for e0, e1 in ev:
            e0.record()
            fn()
            e1.record()
        torch.cuda.synchronize()
        return sorted(e0.elapsed_time(e1) for e0, e1 in ev)[iters // 2] * 1e-3

    lib = L.lib()
    print(f"torch copy_: {nbytes / timed(lambda: dst.copy_(src)) / 1e9:.0f} GB/s")
    for mode in (0, 4, 2, 3, 5, 6, 7):
        lib.sel_tune(49, mode)
        t = timed(lambda: L.call("sel_probe_copy_f4", L.ptr(src), L.ptr(dst), src.numel() // 4, 8 * cus, L.stream()))
        ok = torch.equal(dst, src)
        dst.zero_()
        print(f"mode {mode}: {nbytes / t / 1e9:.0f} GB/s  correct={ok}", flush=True)
    lib.sel_tune(49, 1)
    for blocks in (4 * cus, 8 * cus, 16 * cus, 32 * cus):
        t = timed(lambda: L.call("sel_probe_copy_f4", L.ptr(src), L.ptr(dst), src.numel() // 4, blocks, L.stream()))
        print(f"mode 1 (grid-stride), {blocks} blocks: {nbytes / t / 1e9:.0f} GB/s", flush=True)
    lib.sel_tune(49, 0)


if __name__ == "__main__":
    main()
