"""The denoise-trainer step captured in a HIP graph and replayed.

The reference runs `Trainer._train_step` (trainer/denoise.py:52-84) eagerly:
forward, losses, backward, Adam, scheduler.  Here the step issues ~250 HIP
launches from Python; replayed as one graph, the host issue (several ms per C3
step) leaves the critical path and the GPU runs the launches back to back.

What runs where:
  * in the graph (every replay): the forward, the loss terms and their
    recording, the backward with its deferred weight-gradient reductions, the
    weight packs of the next forward, and the optimizer update — sel.optim.Adam
    with capturable=True, whose step count and learning rate live on the
    device (sel_adam_step_many_dev);
  * on the host after each replay: the LR scheduler (its new rate reaches the
    optimizer's device copy through sync_lr before the next replay), the
    trainer's step counter, progress bar and finish check — the parts of
    _train_step that are host state.
Loss records: while capturing, the trainer's records go to a fixed device
accumulator (one slot per recorded value, allocated before the capture), so
each replay ADDS its values there; `flush_totals()` moves the accumulated sums
into the trainer's own LossTotals (as `total[name] += value` per step would)
and zeroes the accumulator.  The inputs are the fixed device tensors given at
construction (refill them in place to step on new data).

Replays are bit-identical to eager steps of the same trainer
(tests/test_gpu_graph.py): the same kernels run in the same order on the same
buffers.  Single process only: under a process group the gradient all-reduce
stays eager (bench.py replays when world == 1).
"""
import torch

from trainer.trainerGAN import LossTotals


class _CapturedTotals(LossTotals):
    """LossTotals stand-in while capturing: every recorded vector is added
    into consecutive slots of a pre-allocated device accumulator -- all of a
    step's records in one multi-tensor add at the end of the step (one graph
    node instead of one per record)."""

    def __init__(self, acc):
        super().__init__()
        self.acc = acc
        self.names = []
        self.pending = []

    def add(self, name, value):
        if not torch.is_tensor(value):
            raise RuntimeError("graph capture: a host-side loss value cannot be recorded")
        self.add_vector([name], value)

    def add_vector(self, names, value):
        n = len(names)
        if len(self.names) + n > self.acc.numel():
            raise RuntimeError("graph capture: more loss records than accumulator slots")
        self.pending.append((self.acc.narrow(0, len(self.names), n), value.detach().reshape(-1).float()))
        self.names.extend(names)

    def flush(self):
        if self.pending:
            torch._foreach_add_([d for d, _ in self.pending], [v for _, v in self.pending])
            self.pending = []


class GraphedTrainStep:
    """trainer._train_step((x_noisy, x_clean)) captured once, replayed per call."""

    SLOTS = 64

    def __init__(self, trainer, batch, warmup=2):
        self.tr = tr = trainer
        self.batch = batch
        from sel import optim as sel_optim
        opt = tr.optimizer["generator"]
        if not isinstance(opt, sel_optim.Adam) or not all(g["capturable"] for g in opt.param_groups):
            raise ValueError("GraphedTrainStep needs sel.optim.Adam(capturable=True)")
        dev = batch[0].device
        # eager warm-up on a side stream (allocator pools, kernel attributes,
        # one-time plan queries, the optimizer state), as torch's graph capture asks
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(warmup):
                tr._train_step(batch)
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize(dev)

        self.acc = torch.zeros(self.SLOTS, dtype=torch.float32, device=dev)
        rec = _CapturedTotals(self.acc)
        host = dict(totals=tr.total_train_loss, steps=tr.steps, tqdm=tr.tqdm,
                    finish=getattr(tr, "finish_train", False))
        scheds = [s for s in tr.scheduler.values() if s is not None]
        self.graph = torch.cuda.CUDAGraph()
        try:
            tr.total_train_loss = rec
            for s in scheds:
                s.step = lambda *a, **k: None   # host state: stepped after each replay
            with torch.cuda.graph(self.graph):
                tr._train_step(batch)
                rec.flush()
        finally:
            for s in scheds:
                del s.step
            # the capture recorded a step; it ran none: the host state is restored
            tr.total_train_loss = host["totals"]
            tr.steps = host["steps"]
            tr.tqdm = host["tqdm"]
            tr.finish_train = host["finish"]
        self.names = rec.names
        self.opt = opt
        self.scheds = scheds

    def __call__(self):
        self.graph.replay()
        tr = self.tr
        for s in self.scheds:
            s.step()
        self.opt.sync_lr()
        tr.steps += 1
        tr.tqdm.update(1)
        tr._check_train_finish()

    def flush_totals(self):
        """Accumulated loss records of the replays so far -> trainer.total_train_loss."""
        n = len(self.names)
        if n:
            self.tr.total_train_loss.add_vector(self.names, self.acc[:n].clone())
            self.acc.zero_()
