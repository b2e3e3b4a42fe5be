"""The C3 denoise-trainer step replayed as a HIP graph (trainer/graph.py)
against the same step issued eagerly (reference trainer/denoise.py:52-84,
trainer/trainerGAN.py:271-281).

Two trainers from the same seed, both with sel.optim.Adam(capturable=True):
one runs eager steps, the other captures the step once (after the same two
eager warm-up steps) and replays it.  After two replays against two more eager
steps the weights, the Adam moments and step count must be BIT-identical (same
kernels, same order, same buffers' contents), and the recorded losses equal to
float-sum order.  Also: the device-count Adam (sel_adam_step_many_dev) against
the host-constant form, and a scheduler LR change reaching the replayed update.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

B = 4


def _setup(dev, graph):
    import bench
    return bench.c3_setup(dev, B, 1, 0, graph=graph)


def _state(step):
    G = step.generator
    opt = step.trainer.optimizer["generator"]
    out = {k: p.detach().clone() for k, p in G.named_parameters() if p.requires_grad}
    for k, p in G.named_parameters():
        if p.requires_grad:
            st = opt.state[p]
            out[k + ".m"] = st["exp_avg"].clone()
            out[k + ".v"] = st["exp_avg_sq"].clone()
            out[k + ".step"] = torch.as_tensor(st["step"]).detach().clone().cpu()
    return out


def test_graph_replay_bit_identical_to_eager(gpu):
    from sel.convops import precision
    eager = _setup(gpu, graph=False)
    # the eager trainer needs the capturable optimizer too (same update kernels)
    from sel import optim as O
    opt = eager.trainer.optimizer["generator"]
    assert isinstance(opt, O.Adam) and not opt.param_groups[0]["capturable"]
    tr = eager.trainer
    G = eager.generator
    cap = O.Adam([p for p in G.parameters() if p.requires_grad], capturable=True,
                 **{k: opt.param_groups[0][k] for k in ("lr", "betas", "eps", "weight_decay")})
    tr.optimizer["generator"] = cap
    tr.scheduler["generator"] = torch.optim.lr_scheduler.StepLR(cap, step_size=10 ** 9)
    for _ in range(4):          # 2 warm-up + 2 steps, as the graphed trainer below
        eager()
    torch.cuda.synchronize()
    ref = _state(eager)
    ref_loss = {k: float(v) for k, v in tr.total_train_loss.items()}

    graphed = _setup(gpu, graph=True)   # 2 eager warm-up steps, then the capture
    assert hasattr(graphed, "graph")
    graphed()
    graphed()
    torch.cuda.synchronize()
    assert graphed.trainer.steps == 4
    got = _state(graphed)
    for k, v in ref.items():
        assert torch.equal(v, got[k]), k
    graphed.flush_totals()
    got_loss = {k: float(v) for k, v in graphed.trainer.total_train_loss.items()}
    assert set(got_loss) == set(ref_loss)
    for k, v in ref_loss.items():
        assert got_loss[k] == pytest.approx(v, rel=1e-6, abs=1e-9), k
    # one more eager step of the graphed trainer continues from the replayed state
    with precision(torch.bfloat16):
        graphed.eager()
    eager()
    torch.cuda.synchronize()
    ref, got = _state(eager), _state(graphed)
    for k, v in ref.items():
        assert torch.equal(v, got[k]), k


def test_capturable_adam_matches_host_form(gpu):
    """sel_adam_step_many_dev (device count, bias corrections in double on the
    device) against sel_adam_step_many (the host's): the same update up to the
    last float bit of the two constants."""
    from sel import optim as O
    torch.manual_seed(0)
    ps = [torch.randn(n, device=gpu) for n in (1000, 4097, 33)]
    qs = [p.clone() for p in ps]
    a = O.Adam(ps, lr=1e-3, weight_decay=0.01)
    b = O.Adam(qs, lr=1e-3, weight_decay=0.01, capturable=True)
    for it in range(5):
        for p, q in zip(ps, qs):
            g = torch.randn_like(p)
            p.grad, q.grad = g, g.clone()
        a.step()
        b.step()
    torch.cuda.synchronize()
    for p, q in zip(ps, qs):
        assert torch.allclose(p, q, rtol=1e-6, atol=1e-7)
        assert float(b.state[q]["step"]) == 5.0
    # a changed learning rate reaches the device copy
    for g in b.param_groups:
        g["lr"] = 0.0
    before = [q.clone() for q in qs]
    for q in qs:
        q.grad = torch.randn_like(q)
    b.step()
    torch.cuda.synchronize()
    for q, q0 in zip(qs, before):
        assert torch.equal(q, q0)   # lr 0: weight decay enters through the step size too


def test_graph_replay_follows_scheduler(gpu):
    """A StepLR decay between replays changes the replayed update (sync_lr)."""
    g = _setup(gpu, graph=True)
    opt = g.trainer.optimizer["generator"]
    w = next(p for p in g.generator.parameters() if p.requires_grad)
    for grp in opt.param_groups:
        grp["lr"] = 0.0
    opt.sync_lr()
    w0 = w.detach().clone()
    g.graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(w.detach(), w0)      # lr 0 on the device: no update
    for grp in opt.param_groups:
        grp["lr"] = 1e-4
    opt.sync_lr()
    g.graph.replay()
    torch.cuda.synchronize()
    assert not torch.equal(w.detach(), w0)
