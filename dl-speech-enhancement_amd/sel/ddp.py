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
* buckets are all-reduced strictly in index order: a complete bucket waits for
  every lower-indexed one, so all ranks issue the same collectives in the same
  order whatever order their gradients arrive in;
* an autograd final callback launches any bucket left incomplete (parameters
  unused on this rank contribute a zeroed slot) and waits for them all before
  backward() returns.  One float per parameter ("used here") rides in the last
  bucket: a parameter some other rank used gets the averaged gradient, one no
  rank used keeps .grad None (torch DDP with find_unused_parameters).

torch DDP copied every gradient into its bucket and zero-filled buckets each
step (~0.3-0.4 ms per C3 step on one GPU, profiles/r4_ddp_ab.md); this keeps
the one-GPU schedule.  As with torch DDP outside no_sync(), gradients are
not accumulated over several backward calls (each backward averages its
buckets in place): the reference's trainers zero_grad before every backward.
Parameters are broadcast from rank 0 at construction,
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
        # + one "used" flag per parameter after the last gradient: it rides in
        # the last bucket's all-reduce, so which parameters ANY rank used is
        # known without a collective of its own (torch DDP's local_used_map)
        self.nparams = len(params)
        self.flat = torch.zeros(total + self.nparams, dtype=torch.float32, device=dev)
        self.dev_index = dev.index if dev.type == "cuda" else None
        cap = max(1, int(bucket_cap_mb * (1 << 20) / 4))
        self.slots = {}     # id(p) -> (offset, numel, bucket index, weakref(p), flag index)
        self.buckets = []   # [lo, hi, [param ids]]
        off = 0
        for j, p in enumerate(reversed(params)):  # backward order ~ reverse registration order
            if not self.buckets or (self.buckets[-1][1] - self.buckets[-1][0] + p.numel() > cap
                                    and self.buckets[-1][2]):
                self.buckets.append([off, off, []])
            b = self.buckets[-1]
            self.slots[id(p)] = (off, p.numel(), len(self.buckets) - 1, weakref.ref(p), j)
            b[2].append(id(p))
            off += p.numel()
            b[1] = off
        self.buckets[-1][1] = off + self.nparams   # the flags
        self.flags = self.flat.narrow(0, total, self.nparams)
        self._hooks = [p.register_post_accumulate_grad_hook(self._arrived) for p in params]
        self.stats = {"buckets": 0, "copies": 0, "order": []}
        self._reset()

    def _reset(self):
        self.count = [0] * len(self.buckets)
        # streams each bucket's gradients were produced on (the HiFi-GAN
        # discriminator's chains run on side streams, sel.streams: a bucket can
        # hold parameters of several chains)
        self.streams = [[] for _ in self.buckets]
        self.next = 0        # lowest bucket index not yet all-reduced in this backward
        self.used = set()    # ids of the parameters that took a gradient here
        self.works = []
        self.armed = False

    def detach(self):
        """Stop reducing (the module was wrapped again): hooks off, nothing owned."""
        for h in self._hooks:
            h.remove()
        self._hooks = []
        self.slots = {}

    def owns(self, p):
        s = self.slots.get(id(p))
        return s is not None and s[3]() is p

    def view(self, p):
        """A fresh view of p's slot (a new tensor object each call, so that
        AccumulateGrad can keep it as .grad)."""
        off, n = self.slots[id(p)][:2]
        return self.flat.narrow(0, off, n).view(p.shape)

    def _arrived(self, p):
        if p.grad is None:  # an undefined gradient (e.g. a frozen pass): not an arrival
            return
        if not self.armed:
            self.armed = True
            self.stats["order"] = []   # this backward's launch order only (bounded)
            torch.autograd.Variable._execution_engine.queue_callback(self._finish)
        off, n, bi = self.slots[id(p)][:3]
        g = p.grad
        if g.data_ptr() != self.flat.data_ptr() + 4 * off or g.numel() != n or g.dtype != torch.float32:
            # a gradient from outside the sel weight-gradient ops: into the slot
            v = self.view(p)
            v.copy_(g)
            p.grad = v
            self.stats["copies"] += 1
        # the stream this gradient was produced on (AccumulateGrad runs on it);
        # the raw (id, device, type) triple: this hook runs once per parameter
        # per backward, and torch.cuda.current_stream() would build a Stream
        # object each time on the host's critical path
        if self.dev_index is not None:
            st = torch._C._cuda_getCurrentStream(self.dev_index)
            if st not in self.streams[bi]:
                self.streams[bi].append(st)
        if id(p) not in self.used:
            self.used.add(id(p))
            self.count[bi] += 1
        # all-reduces leave in bucket-index order on every rank, whatever order
        # the buckets complete in (RCCL matches collectives by issue order)
        while self.next < len(self.buckets) and self.count[self.next] == len(self.buckets[self.next][2]):
            self._launch(self.next)

    def _launch(self, bi):
        assert bi == self.next
        lo, hi, ids = self.buckets[bi]
        if bi == len(self.buckets) - 1 and self.world > 1:
            if len(self.used) == self.nparams:
                self.flags.fill_(1.0)
            else:
                f = torch.zeros(self.nparams, dtype=torch.float32)
                for i in self.used:
                    f[self.slots[i][4]] = 1.0
                self.flags.copy_(f, non_blocking=False)
        # the reductions, the 1/W and the all-reduce go on the current stream:
        # it first waits for every other stream that wrote gradients of this
        # bucket (without it a bucket spanning two discriminator chains was
        # read while the other chain's weight-gradient kernels still ran)
        if self.dev_index is not None:
            cur = torch._C._cuda_getCurrentStream(self.dev_index)
            others = [st for st in self.streams[bi] if st != cur]
            if others:
                cs = torch.cuda.Stream(stream_id=cur[0], device_index=cur[1], device_type=cur[2])
                for st in others:
                    cs.wait_stream(torch.cuda.Stream(stream_id=st[0], device_index=st[1], device_type=st[2]))
        ps = [self.slots[i][3]() for i in ids]
        CO.flush_params([p for p in ps if p is not None])
        sl = self.flat[lo:hi]
        if self.world > 1:
            self._scale(sl)
            self.works.append(dist.all_reduce(sl, group=self.pg, async_op=True))
        self.next += 1
        self.stats["buckets"] += 1
        self.stats["order"].append(bi)

    def _scale(self, sl):
        """Pre-divide a bucket by W so the all-reduce SUM is the average."""
        sl.div_(self.world)

    def _finish(self):
        unused = [i for i in self.slots if i not in self.used]
        for i in unused:  # parameters that took no gradient here contribute zeros
            p = self.slots[i][3]()
            if p is not None and p.grad is not None:
                continue   # a gradient kept from an earlier backward stays (see the class note)
            off, n = self.slots[i][:2]
            self.flat.narrow(0, off, n).zero_()
        while self.next < len(self.buckets):
            self._launch(self.next)
        for w in self.works:
            w.wait()
        if unused and self.world > 1:
            # a parameter another rank used gets the average (this rank's zeros
            # included), as under torch DDP; one nobody used keeps .grad None
            flags = self.flags.tolist()
            for i in unused:
                p = self.slots[i][3]()
                if p is not None and flags[self.slots[i][4]] > 0:
                    p.grad = self.view(p)
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
        CO.register_grad_buckets(self.reducer)   # (detaches an older reducer of these parameters)

    def forward(self, *args, **kwargs):
        return self.module(*args, **kwargs)

    def state_dict(self, *args, **kwargs):
        return self.module.state_dict(*args, **kwargs)

    def load_state_dict(self, state_dict, strict=True, **kwargs):
        return self.module.load_state_dict(state_dict, strict=strict, **kwargs)
