"""Independent HIP-kernel chains on side streams (the HiFi-GAN discriminator's
8 sub-discriminators, models/vocoder/HiFiGAN.py:380-395).

A sub-discriminator's layers are launches of a few hundred 256-row tiles
(C5: the MPD's 512 / 1024-wide layers make 150-300 tiles for 256 CUs), so each
one leaves CUs idle in its last round; its weight-gradient reductions and
loss kernels are small launches.  The 8 chains share no data but the input
waveform, so running them on side streams lets one chain's launches fill the
CUs another leaves idle.  Kernels, launch order per chain and every result
are unchanged (each chain's launches stay in order on its stream; no kernel
has cross-launch atomics), so the outputs are bit-identical to the serial
form.  Autograd runs each chain's backward on the stream of its forward and
synchronises the streams where gradients cross them (torch's stream semantics
of backward passes).

SEL_D_STREAMS = number of side streams (default 8: one per chain; 0 =
everything on the current stream).  Measured at C5, alternating in one call:
8 streams 35.2 / 35.4 ms median, 4 streams 36.1 / 35.8, 2 streams 35.8 / 35.8,
serial 41.8 (an earlier call); raising GPU_MAX_HW_QUEUES from the box's 4 to 8 made the step
48-54 ms.  Launching D(target) on the side streams before the generator
forward (it needs neither) measured neutral (35.8 vs 35.9-36.1 ms median).
"""
import os

import torch

_POOL = {}


def side_streams(device):
    n = int(os.environ.get("SEL_D_STREAMS", "8"))
    if n <= 0 or device.type != "cuda":
        return []
    key = (device.index, n)
    if key not in _POOL:
        _POOL[key] = [torch.cuda.Stream(device=device) for _ in range(n)]
    return _POOL[key]


def _tensors(obj):
    if isinstance(obj, torch.Tensor):
        yield obj
    elif isinstance(obj, (list, tuple)):
        for o in obj:
            yield from _tensors(o)


def run_concurrent(calls, inputs):
    """Run zero-argument callables `calls` (chain i on side stream i mod n) and
    return their results; `inputs` are the tensors of the current stream they
    read.  The current stream waits for every side stream before it goes on,
    and the allocator is told which streams use which blocks (record_stream),
    so no block is reused while another stream may still read it."""
    dev = inputs[0].device
    ss = side_streams(dev)
    if not ss:
        return [c() for c in calls]
    main = torch.cuda.current_stream(dev)
    used = ss[:len(calls)]
    for s in used:
        s.wait_stream(main)
    outs = []
    for i, c in enumerate(calls):
        with torch.cuda.stream(used[i % len(used)]):
            outs.append(c())
    for s in used:
        main.wait_stream(s)
    for t in inputs:
        for s in used:
            t.record_stream(s)
    for t in _tensors(outs):
        t.record_stream(main)
    return outs
