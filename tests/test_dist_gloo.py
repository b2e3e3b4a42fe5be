"""World-size-2 data-parallel tests on CPU (gloo, 127.0.0.1).

Cover the host logic of sel/dist.py: equal sharding of the global batch, the
batch-global add_noise exchange (per-rank sums -> all-reduce -> mix; the two
device kernels are replaced by their oracle math so only the exchange is under
test here — tests/test_gpu_glue.py checks the kernels themselves), and that the
DDP wrapper's averaged gradients equal the single-process full-batch gradient
for a mean loss (the property the denoise step relies on, sel/dist.py docstring).
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import ref_ops as R

WORLD = 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, port, fn, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(WORLD), LOCAL_RANK=str(rank))
    try:
        from sel import dist as D
        D.init_from_env(backend="gloo")
        res = fn(rank)
        # numpy, not tensors: torch's shared-memory handles die with the child
        res = [t.numpy() for t in res] if isinstance(res, list) else res.numpy()
        q.put((rank, res))
    except Exception as e:  # pragma: no cover - surfaced by the parent
        q.put((rank, e))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def _run(fn):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, fn, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for r, v in out.items():
        if isinstance(v, Exception):
            raise v
    conv = lambda v: [torch.from_numpy(a) for a in v] if isinstance(v, list) else torch.from_numpy(v)
    return {r: conv(v) for r, v in out.items()}


def _global_batch():
    g = torch.Generator().manual_seed(7)
    speech = torch.randn(4, 1, 4800, generator=g, dtype=torch.float64).float()
    noise = 0.3 * torch.randn(4, 1, 4800, generator=g, dtype=torch.float64).float()
    return speech, noise


def _add_noise_case(rank):
    from sel import dist as D

    def local_sumsq(s, n):  # oracle math of sel_sumsq2
        return torch.stack([(s.double() ** 2).sum(), (n.double() ** 2).sum()])

    def mix(s, n, sums, snr):  # oracle math of sel_mix_noise
        import math
        scale = math.exp(snr / 10) * math.sqrt(float(sums[1])) / math.sqrt(float(sums[0]))
        return ((scale * s.double() + n.double()) / 2).float()

    D._local_sumsq, D._mix = local_sumsq, mix
    speech, noise = _global_batch()
    return D.add_noise_global(D.shard(speech), D.shard(noise), 5.0)


def test_add_noise_global_matches_single_device():
    out = _run(_add_noise_case)
    speech, noise = _global_batch()
    ref = R.add_noise(speech.double(), noise.double(), 5.0).float()
    got = torch.cat([out[0], out[1]])
    torch.testing.assert_close(got, ref, rtol=1e-6, atol=1e-6)
    # rank-local norms would differ: the exchange is load-bearing
    loc = torch.cat([R.add_noise(speech[:2], noise[:2], 5.0), R.add_noise(speech[2:], noise[2:], 5.0)])
    assert (loc - ref).abs().max() > 1e-3


def _tiny_model():
    torch.manual_seed(3)
    return torch.nn.Sequential(torch.nn.Conv1d(1, 8, 7, padding=3), torch.nn.ELU(), torch.nn.Conv1d(8, 1, 3, padding=1))


def _batch():
    g = torch.Generator().manual_seed(11)
    return torch.randn(4, 1, 256, generator=g), torch.randn(4, 1, 256, generator=g)


def _ddp_case(rank):
    from sel import dist as D
    m = D.wrap_ddp(_tiny_model())
    x, y = _batch()
    loss = torch.nn.functional.l1_loss(m(D.shard(x)), D.shard(y))
    loss.backward()
    return [p.grad.clone() for p in m.parameters()]


def test_ddp_grad_equals_full_batch():
    out = _run(_ddp_case)
    m = _tiny_model()
    x, y = _batch()
    torch.nn.functional.l1_loss(m(x), y).backward()
    for r in range(WORLD):
        for g, p in zip(out[r], m.parameters()):
            torch.testing.assert_close(g, p.grad, rtol=1e-5, atol=1e-6)


def _buckets_case(rank):
    """sel.ddp with one-parameter buckets (bucket_cap_mb tiny), an unused
    parameter and two backward passes: every bucket all-reduced in order,
    the unused parameter's .grad left None."""
    from sel.ddp import SelDDP

    class WithUnused(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.net = _tiny_model()
            self.extra = torch.nn.Linear(2, 2)  # never used: its bucket is launched by the final callback

        def forward(self, x):
            return self.net(x)
    model = WithUnused()
    m = SelDDP(model, bucket_cap_mb=1e-6)
    assert len(m.reducer.buckets) == len(list(model.parameters()))
    x, y = _batch()
    out = []
    for it in range(2):
        for p in model.parameters():
            p.grad = None
        loss = torch.nn.functional.l1_loss(m(D_shard(x)), D_shard(y)) * (it + 1)
        loss.backward()
        assert model.extra.weight.grad is None and model.extra.bias.grad is None
        out += [p.grad.clone() for p in model.parameters() if p.grad is not None]
    assert m.reducer.stats["buckets"] == 2 * len(m.reducer.buckets)
    # the state dict has the wrapped module's keys (no "module." prefix)
    assert set(m.state_dict()) == set(model.state_dict())
    return out


def D_shard(t):
    from sel import dist as D
    return D.shard(t)


def test_sel_ddp_buckets_average_like_full_batch():
    out = _run(_buckets_case)
    m = _tiny_model()
    x, y = _batch()
    ref = []
    for it in range(2):
        m.zero_grad(set_to_none=True)
        (torch.nn.functional.l1_loss(m(x), y) * (it + 1)).backward()
        ref += [p.grad.clone() for p in m.parameters()]
    for r in range(WORLD):
        assert len(out[r]) == len(ref)
        for g, gr in zip(out[r], ref):
            torch.testing.assert_close(g, gr, rtol=1e-5, atol=1e-6)


class _Branches(torch.nn.Module):
    """Two independent branches (their gradients arrive in the reverse order of
    their forward), a head used on rank 0 only and a layer no rank uses."""

    def __init__(self):
        super().__init__()
        torch.manual_seed(5)
        self.a = torch.nn.Conv1d(1, 4, 5, padding=2)
        self.b = torch.nn.Conv1d(1, 6, 3, padding=1)
        self.head = torch.nn.Linear(4, 3)
        self.never = torch.nn.Linear(2, 2)

    def loss(self, x, y, rank):
        if rank == 0:
            ya, yb = self.a(x), self.b(x)
        else:  # the other forward order: the backward completes buckets differently
            yb, ya = self.b(x), self.a(x)
        loss = torch.nn.functional.l1_loss(ya.mean(1, keepdim=True) + yb.mean(1, keepdim=True), y)
        if rank == 0:
            loss = loss + 0.1 * self.head(ya.mean(-1)).square().mean()
        return loss


def _order_case(rank):
    """sel.ddp: the ranks' gradients arrive in different orders, yet every rank
    issues its all-reduces in bucket-index order (one-parameter buckets of
    different sizes: an order mismatch would pair unequal tensors); the head,
    used on rank 0 only, gets the average on BOTH ranks; the unused layer keeps
    .grad None; a second wrap of the same module detaches the first reducer."""
    from sel.ddp import SelDDP
    from sel import dist as D
    model = _Branches()
    first = SelDDP(model, bucket_cap_mb=1e-6)
    m = SelDDP(model, bucket_cap_mb=1e-6)          # wrapped again: `first` is detached
    assert not first.reducer.slots and not first.reducer._hooks
    arrivals = []
    for name, p in model.named_parameters():
        p.register_post_accumulate_grad_hook(lambda p, name=name: arrivals.append(name))
    x, y = _batch()
    model.zero_grad(set_to_none=True)
    model.loss(D.shard(x), D.shard(y), rank).backward()
    assert m.reducer.stats["order"] == list(range(len(m.reducer.buckets)))
    assert model.never.weight.grad is None and model.never.bias.grad is None
    assert model.head.weight.grad is not None
    first_a = min(i for i, n in enumerate(arrivals) if n.startswith("a."))
    first_b = min(i for i, n in enumerate(arrivals) if n.startswith("b."))
    names = [n for n, p in model.named_parameters() if p.grad is not None]
    return [torch.tensor([first_a < first_b])] + [p.grad.clone() for n, p in model.named_parameters()
                                                    if p.grad is not None] + [torch.tensor(len(names))]


def test_sel_ddp_ordered_buckets_and_unused_parameters():
    out = _run(_order_case)
    # the two ranks really completed the branches in different orders
    assert bool(out[0][0]) != bool(out[1][0])
    model = _Branches()
    x, y = _batch()
    ((model.loss(x[:2], y[:2], 0) + model.loss(x[2:], y[2:], 1)) / WORLD).backward()
    ref = [p.grad for n, p in model.named_parameters() if p.grad is not None]
    for r in range(WORLD):
        assert int(out[r][-1]) == len(ref)
        for g, gr in zip(out[r][1:-1], ref):
            torch.testing.assert_close(g, gr, rtol=1e-5, atol=1e-7)


def _shard_case(rank):
    from sel import dist as D
    t = torch.arange(8)
    assert D.rank_world() == (rank, WORLD)
    return D.shard(t)


def test_shard_disjoint_cover():
    out = _run(_shard_case)
    assert torch.equal(torch.cat([out[0], out[1]]), torch.arange(8))


def test_shard_rejects_ragged():
    from sel import dist as D
    with pytest.raises(ValueError):
        D.shard(torch.arange(5), rank=0, world=2)


def _mags():
    g = torch.Generator().manual_seed(21)
    xm = torch.rand(4, 31, 17, generator=g, dtype=torch.float64) + 0.05
    ym = torch.rand(4, 31, 17, generator=g, dtype=torch.float64) + 0.05
    return xm, ym


def _sc_case(rank):
    """Rank-local partial sums (the kernel's sel_mag_pair_sums, restated) ->
    sel.dist.global_loss_sums -> SC / log-mag and the per-rank gradient the
    autograd op back-propagates (the sel_stft_loss_coef formula with grad_scale)."""
    from sel import dist as D
    xm, ym = _mags()
    x, y = D.shard(xm), D.shard(ym)
    sums = torch.stack([((y - x) ** 2).sum(), (y ** 2).sum(), (torch.log(y) - torch.log(x)).abs().sum()])
    sums_g, n_g, scale = D.global_loss_sums(sums, x.numel())
    # the global count stays on device (sums_g[3]); n = 0 tells the finishing
    # kernels to read it there (no host sync)
    assert n_g == 0 and sums_g.shape == (4,) and scale == WORLD
    assert sums_g[3].item() == xm.numel()
    n_g = sums_g[3]
    n1, n2 = sums_g[0].sqrt(), sums_g[1].sqrt()
    sc, mag = n1 / n2, sums_g[2] / n_g
    # d/dx of sc and mag w.r.t. this shard, times grad_scale (stft_loss_coef + mag_pair_bwd)
    gx = scale * ((x - y) / (n1 * n2) + torch.sign(torch.log(x) - torch.log(y)) / x / n_g)
    return [torch.stack([sc, mag]), gx]


def test_spectral_convergence_is_global_under_dp():
    """losses/stft_loss.py:56 is a ratio of GLOBAL Frobenius norms: under data
    parallelism the exchanged sums give the single-device value on the global
    batch, and the DDP-averaged gradient (grad/W per shard) equals the
    single-device gradient."""
    out = _run(_sc_case)
    xm, ym = _mags()
    xr = xm.clone().requires_grad_(True)
    sc, mag = R.spectral_convergence(xr, ym), R.log_stft_magnitude(xr, ym)
    (sc + mag).backward()
    for r in range(WORLD):
        torch.testing.assert_close(out[r][0], torch.stack([sc, mag]).detach(), rtol=1e-12, atol=0)
    got = torch.cat([out[0][1], out[1][1]]) / WORLD
    torch.testing.assert_close(got, xr.grad, rtol=1e-10, atol=1e-14)
    # rank-local SC (no exchange) differs: the exchange is load-bearing
    loc = R.spectral_convergence(xm[:2], ym[:2])
    assert abs(loc.item() - sc.item()) > 1e-4


def test_adam_factory_falls_back_to_torch_off_gpu():
    """sel.optim.adam builds torch's Adam for CPU parameters (and for the options
    sel.optim.Adam refuses); on the GPU path it is sel.optim.Adam."""
    import torch
    from sel import optim as O
    p = [torch.zeros(3, requires_grad=True)]
    assert type(O.adam(p, lr=1e-3, fused=False)) is torch.optim.Adam
    with pytest.raises(NotImplementedError):
        O.Adam(p, lr=1e-3, amsgrad=True)
