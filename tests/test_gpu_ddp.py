"""The data-parallel PRODUCT step, executed: two ranks on the box's one GPU.

Each rank is a fresh child process (tests/ddp_product_worker.py; the pytest
process is never exec'ed) in a world-size-2 gloo process group over CUDA
tensors.  RCCL cannot place two ranks on one device; gloo can, and everything
above the backend is what bench.py / train_denoise.py run over RCCL on 8 GPUs:
DDP's bucket hooks on the HIP autograd ops, the deferred weight-gradient
reductions run per gradient bucket by the sel reducer (sel/ddp.py, convops
flush_params; asserted to have run), the packed-weight
refresh after the DDP-averaged Adam step, the batch-global add_noise exchange
(sel.dist.add_noise_global), the spectral-convergence exchange through the real
STFT-loss autograd op (sel.dist.global_loss_sums, losses/stft_loss.py:56), the
frozen-D generator pass on the unwrapped discriminator and the single
concatenated-batch D step under DDP (train_denoise.py DenoiseStep), and the
global SNR surrogate (train_denoise._global_snr_term).

Reference: the same step in THIS process without a process group, on the
concatenated global batch (data parallelism must reproduce the
single-device step).  Loss terms: the mean over ranks of each rank's value
equals the single-device value (every term is a shard mean or an exchanged
global quantity) to 1e-5.  Weights after two Adam steps: the bounds of
test_gpu_glue.py (<= 2% of weights flip their update direction, <= 10%
norm-wise update error; the per-rank gradient sums run in another order).
"""
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
WORKER = os.path.join(HERE, "ddp_product_worker.py")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_ranks(case, tmp_path, world=2, timeout=240):
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK="0", LOCAL_WORLD_SIZE=str(world),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
        log = open(tmp_path / f"rank{r}.log", "w")
        procs.append((subprocess.Popen([sys.executable, "-u", WORKER, case, str(tmp_path / f"rank{r}.pt")],
                                       env=env, stdout=log, stderr=subprocess.STDOUT), log))
    rcs = []
    try:
        for p, _ in procs:
            rcs.append(p.wait(timeout=timeout))
    finally:
        for p, log in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
            log.close()
    if any(rcs):
        logs = "\n".join((tmp_path / f"rank{r}.log").read_text()[-3000:] for r in range(world))
        raise AssertionError(f"ranks exited {rcs}:\n{logs}")
    return [torch.load(tmp_path / f"rank{r}.pt", weights_only=True) for r in range(world)]


def _update_check(p0, ref, got, lr):
    """(#weights whose update moved > lr/2 from the reference's, #weights,
    squared update error, squared reference update)."""
    du_ref = ref.double() - p0.double()
    du = got.double() - p0.double()
    return (((du - du_ref).abs() > 0.5 * lr).sum().item(), du.numel(), ((du - du_ref) ** 2).sum().item(),
            (du_ref ** 2).sum().item())


@pytest.mark.parametrize("case", ["pqc", "c3", "bench", "gan"])
def test_ddp_product_step_matches_single_process(gpu, case, tmp_path):
    import ddp_product_worker as W
    ranks = _run_ranks(case, tmp_path)
    assert [tuple(r["rank_world"]) for r in ranks] == [(0, 2), (1, 2)]
    assert all(r["deferred_pending"] == 0 for r in ranks)
    if case in ("pqc", "c3", "bench"):
        # the generator's weight-gradient reductions were deferred under the
        # process group and run by the sel reducer, per bucket
        for r in ranks:
            assert r["ddp_stats"]["jobs"] > 0 and r["ddp_stats"]["bucket_flushes"] > 0, r["ddp_stats"]
    # DDP keeps the replicas identical
    for k, v in ranks[0]["params"].items():
        assert torch.equal(v, ranks[1]["params"][k]), k
    # initial weights: the same seeded construction, in this process
    torch.manual_seed(0)
    ref = W.run_case(case, gpu)
    torch.cuda.synchronize()
    # bench: the bf16 conv kernels are chosen by row count (sel fwd4_choice:
    # 8 clips per rank put the 256-wide layers at 3,200 rows, under the tiles the
    # 16-clip process uses), so the two runs round differently in bf16; 1e-3
    # bounds that (measured 2.6e-4 on the mel loss before any update).  The other
    # cases run the same kernels on both sides: 1e-5.
    rtol = 1e-3 if case == "bench" else 1e-5
    for s, ref_s in enumerate(ref["steps"]):
        for name, v in ref_s.items():
            got = sum(r["steps"][s][name] for r in ranks) / len(ranks)
            assert abs(got - v) <= rtol * abs(v) + 1e-7, (case, s, name, got, v, [r["steps"][s][name] for r in ranks])
    # the exchanged terms are load-bearing: without them the rank values would differ
    if case == "pqc":
        sc = [r["steps"][0]["train/spectral_convergence_loss"] for r in ranks]
        assert sc[0] == pytest.approx(sc[1], rel=1e-6), sc  # global SC: the same scalar on both ranks
    # weight updates of two Adam steps (lr: generator 1e-4, discriminator 2e-4)
    p0 = _initial_params(case, gpu)
    groups = {}
    for k, v in ref["params"].items():
        lr = 2e-4 if k.startswith("D.") else 1e-4
        a, n, num, den = _update_check(p0[k], v, ranks[0]["params"][k], 2 * lr)
        g = groups.setdefault(k.split(".")[0] if case == "gan" else "G", [0, 0, 0.0, 0.0])
        g[0] += a
        g[1] += n
        g[2] += num
        g[3] += den
    # Adam's first steps move each weight by about +-lr whatever the gradient's
    # size, so a weight whose tiny gradient changes sign costs (4 lr)^2 of
    # squared error against (2 lr)^2 of update: 0.25% sign changes alone give a
    # 10% norm-wise error.  The bench case (16 clips, full width, bf16, kernels
    # chosen by row count, 10k RVQ argmins whose near-ties flip with the
    # rounding) runs at 0.11: bounded at 0.15, with the 2% flip bound unchanged.
    nbound = 0.15 if case == "bench" else 0.10
    for name, (flips, tot, num, den) in groups.items():
        assert tot > 0 and flips <= 0.02 * tot, (case, name, flips, tot)
        assert (num / den) ** 0.5 <= nbound, (case, name, (num / den) ** 0.5)


def _initial_params(case, dev):
    """The seeded initial weights of run_case (same construction order)."""
    import warnings
    import ddp_product_worker as W
    from sel import configs
    torch.manual_seed(0)
    if case == "bench":
        import bench
        from models.autoencoder.AudioDec import Generator
        torch.manual_seed(93)   # bench.c3_setup's seed
        G = Generator(**configs.get(bench.C3_CONFIG)["generator_params"])
        return {k: p.detach().clone() for k, p in G.named_parameters()}
    if case in ("pqc", "c3"):
        from models.autoencoder.AudioDec import Generator
        cfg = configs.get("symAD_libritts_24000_hop300")
        G = Generator(**dict(cfg["generator_params"], **(W.GP if case == "pqc" else {})))
        return {k: p.detach().clone() for k, p in G.named_parameters()}
    from models.autoencoder_without_PQC.AudioDec import Generator
    from models.vocoder.HiFiGAN import Discriminator
    cfg = configs.get("symAD_vctk_48000_hop300")
    G = Generator(**dict(cfg["generator_params"], **W.GP))
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        Dm = Discriminator(**W.D_PARAMS)
    out = {f"G.{k}": p.detach().clone() for k, p in G.named_parameters()}
    out.update({f"D.{k}": p.detach().clone() for k, p in Dm.named_parameters()})
    return out
