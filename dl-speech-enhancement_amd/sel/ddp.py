"""Data-parallel gradient averaging for the sel hot path (the role of torch's
DistributedDataParallel, built around the deferred weight-gradient reductions
of sel.convops).

One process per GPU (bench.py / train_denoise.py under torch.distributed.run),
RCCL all-reduce over xGMI.  The trainable parameters' gradients live in ONE
flat fp32 buffer, cut into ~4 MB buckets in backward order:

* the sel weight-gradient ops return a fresh view of the parameter's slot as
  its gradient (AccumulateGrad keeps that very tensor as .grad: no copy), and
  their deferred reductions (sel_wgrad_finish_many) write into the slots;
* a post-accumulate-grad hook per parameter counts the bucket's arrivals (and
  copies a gradient that some other op produced into its slot, as DDP does);
* when a bucket is complete, its pending reductions run as ONE launch, the
  slice is scaled by 1/W and all-reduced asynchronously (RCCL overlaps the rest
  of the backward);
* an autograd final callback launches any bucket left incomplete (parameters
  unused in this backward: their slots are zeroed, .grad stays None) in bucket
  order, so every rank issues the same collectives, and waits for them all
  before backward() returns.

torch DDP copied every gradient into its bucket and zero-filled buckets each
step (~0.3-0.4 ms per C3 step on one GPU, profiles/r4_ddp_ab.md); this keeps
the one-GPU schedule.  Parameters are broadcast from rank 0 at construction,
as DDP does; buffers are not (broadcast_buffers=False in every call site).
"""
import weakref

import torch
import torch.distributed as dist

from . import convops as CO


class GradBuckets:
    def __init__(self, params, bucket_cap_mb=4.0, process_group=None):
        self.pg = process_group
        self.world = dist.get_world_size(process_group)
        params = [p for p in params if p.requires_grad]
        if not params:
            raise ValueError("no trainable parameters")
        dev = params[0].device
        if any(p.device != dev or p.dtype != torch.float32 for p in params):
            raise ValueError("GradBuckets: fp32 parameters on one device")
        total = sum(p.numel() for p in params)
        self.flat = torch.zeros(total, dtype=torch.float32, device=dev)
        cap = max(1, int(bucket_cap_mb * (1 << 20) / 4))
        self.slots = {}     # id(p) -> (offset, numel, bucket index, weakref(p))
        self.buckets = []   # [lo, hi, [param ids]]
        off = 0
        for p in reversed(params):  # backward order ~ reverse registration order
            if not self.buckets or (self.buckets[-1][1] - self.buckets[-1][0] + p.numel() > cap
                                    and self.buckets[-1][2]):
                self.buckets.append([off, off, []])
            b = self.buckets[-1]
            self.slots[id(p)] = (off, p.numel(), len(self.buckets) - 1, weakref.ref(p))
            b[2].append(id(p))
            off += p.numel()
            b[1] = off
        self._hooks = [p.register_post_accumulate_grad_hook(self._arrived) for p in params]
        self.stats = {"buckets": 0, "copies": 0}
        self._reset()

    def _reset(self):
        self.count = [0] * len(self.buckets)
        self.launched = [False] * len(self.buckets)
        self.works = []
        self.armed = False

    def owns(self, p):
        s = self.slots.get(id(p))
        return s is not None and s[3]() is p

    def view(self, p):
        """A fresh view of p's slot (a new tensor object each call, so that
        AccumulateGrad can keep it as .grad)."""
        off, n, _, _ = self.slots[id(p)]
        return self.flat.narrow(0, off, n).view(p.shape)

    def _arrived(self, p):
        if p.grad is None:  # an undefined gradient (e.g. a frozen pass): not an arrival
            return
        if not self.armed:
            self.armed = True
            torch.autograd.Variable._execution_engine.queue_callback(self._finish)
        off, n, bi, _ = self.slots[id(p)]
        g = p.grad
        if g.data_ptr() != self.flat.data_ptr() + 4 * off or g.numel() != n or g.dtype != torch.float32:
            # a gradient from outside the sel weight-gradient ops: into the slot
            v = self.view(p)
            v.copy_(g)
            p.grad = v
            self.stats["copies"] += 1
        self.count[bi] += 1
        if self.count[bi] == len(self.buckets[bi][2]):
            self._launch(bi)

    def _launch(self, bi):
        lo, hi, ids = self.buckets[bi]
        ps = [self.slots[i][3]() for i in ids]
        CO.flush_params([p for p in ps if p is not None])
        sl = self.flat[lo:hi]
        if self.world > 1:
            sl.div_(self.world)
            self.works.append(dist.all_reduce(sl, group=self.pg, async_op=True))
        self.launched[bi] = True
        self.stats["buckets"] += 1

    def _finish(self):
        for bi, (lo, hi, ids) in enumerate(self.buckets):
            if self.launched[bi]:
                continue
            for i in ids:  # parameters that took no gradient in this backward
                p = self.slots[i][3]()
                if p is not None and p.grad is None:
                    off, n, _, _ = self.slots[i]
                    self.flat.narrow(0, off, n).zero_()
            self._launch(bi)
        for w in self.works:
            w.wait()
        self._reset()


class SelDDP(torch.nn.Module):
    """DistributedDataParallel's interface for the sel hot path: forward is the
    wrapped module's, .module is the wrapped module, state_dict() / load_state_dict()
    are the wrapped module's (the reference's keys, no "module." prefix)."""

    def __init__(self, module, bucket_cap_mb=4.0, process_group=None):
        super().__init__()
        self.module = module
        if dist.get_world_size(process_group) > 1:
            with torch.no_grad():
                for p in module.parameters():
                    dist.broadcast(p.data, src=dist.get_global_rank(process_group, 0) if process_group else 0,
                                   group=process_group)
        self.reducer = GradBuckets(module.parameters(), bucket_cap_mb, process_group)
        CO.register_grad_buckets(self.reducer)

    def forward(self, *args, **kwargs):
        return self.module(*args, **kwargs)

    def state_dict(self, *args, **kwargs):
        return self.module.state_dict(*args, **kwargs)

    def load_state_dict(self, state_dict, strict=True, **kwargs):
        return self.module.load_state_dict(state_dict, strict=strict, **kwargs)
