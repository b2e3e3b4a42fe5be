"""CPU checks of host-side logic that needs no GPU: the packed-weight cache's
staleness signals, the bench launcher, the trainer checkpoint layout and the
data-parallel sampler epochs."""
import os
import sys

import pytest
import torch

from conftest import REPO


def _entry(cache, w, kind=0):
    from sel import convops as CO
    e = CO._PackEntry()
    e.wref, e.pid, e.kind, e.stride, e.dtype = __import__("weakref").ref(w), id(w), kind, 1, torch.float32
    e.version, e.wp, e.wd = w._version, None, None
    key = (w.data_ptr(), kind, 1, torch.float32, tuple(w.shape), w.device)
    cache._entries[key] = e
    cache._by_param.setdefault(id(w), []).append(key)
    return e


@pytest.mark.parametrize("kw", [dict(fused=True), dict(foreach=True), dict(foreach=False)])
def test_pack_cache_goes_stale_after_every_adam_flavour(kw):
    """Fused Adam updates parameters without bumping ``_version``; the global
    optimizer post-step hook must mark their packs stale anyway."""
    from sel import convops as CO
    w = torch.nn.Parameter(torch.randn(4, 3, 7))
    other = torch.nn.Parameter(torch.randn(4, 3, 7))
    e = _entry(CO.PACKS, w)
    e2 = _entry(CO.PACKS, other)
    try:
        opt = torch.optim.Adam([w], lr=1e-2, **kw)
        w.grad = torch.randn_like(w)
        opt.step()
        assert e.version is None or e.version != w._version
        # a parameter the optimizer does not own keeps its pack
        assert e2.version == other._version
    finally:
        CO.PACKS.invalidate()


def test_fused_adam_really_skips_the_version_bump():
    """Documents why the hook exists: if torch ever bumps the version in fused
    Adam this test fails and the hook becomes belt-and-braces only."""
    w = torch.nn.Parameter(torch.randn(8))
    v0 = w._version
    opt = torch.optim.Adam([w], lr=1e-2, fused=True)
    w.grad = torch.randn_like(w)
    before = w.detach().clone()
    opt.step()
    assert not torch.equal(before, w.detach())
    assert w._version == v0


def test_bench_launch_cmd_runs_n_ranks_of_itself():
    sys.path.insert(0, REPO)
    import bench
    cmd = bench.launch_cmd(8, 29555, ["--gpus", "8", "--steps", "20"])
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--master-addr=127.0.0.1" in cmd and "--master-port=29555" in cmd
    assert cmd[-5:] == [os.path.join(REPO, "bench.py"), "--gpus", "8", "--steps", "20"]


def test_bench_launcher_starts_world_size_ranks(tmp_path):
    """The relaunch command really yields WORLD_SIZE = N ranks with RANK 0..N-1
    (gloo, CPU): run the same torch.distributed.run line on a probe script."""
    import subprocess
    probe = tmp_path / "probe.py"
    probe.write_text("import os, torch.distributed as d\n"
                     "d.init_process_group('gloo')\n"
                     "print('RANK', os.environ['RANK'], os.environ['WORLD_SIZE'], d.get_world_size(), flush=True)\n"
                     "d.destroy_process_group()\n")
    sys.path.insert(0, REPO)
    import bench
    import socket
    # loopback for gloo's own sockets; one retry on a fresh port (the probe port
    # is released before torch.distributed.run binds it, so another process can
    # take it in between: a rendezvous failure, not a launcher one)
    env = dict(os.environ, GLOO_SOCKET_IFNAME="lo")
    for attempt in range(2):
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        cmd = bench.launch_cmd(2, port, [])
        cmd[-1] = str(probe)
        out = subprocess.run(cmd, capture_output=True, text=True, timeout=120, env=env)
        if out.returncode == 0:
            break
    assert out.returncode == 0, out.stderr[-2000:]
    lines = sorted(l for l in out.stdout.splitlines() if l.startswith("RANK"))
    assert lines == ["RANK 0 2 2", "RANK 1 2 2"], out.stdout


def test_set_epoch_reshuffles_distributed_shards():
    """every epoch must draw a new DistributedSampler order."""
    from torch.utils.data import DataLoader, DistributedSampler
    from dataloader.data_utils import set_epoch
    ds = list(range(64))
    s = DistributedSampler(ds, num_replicas=2, rank=0, shuffle=True, seed=82, drop_last=True)
    dl = DataLoader(ds, batch_size=4, sampler=s)
    plain = DataLoader(ds, batch_size=4, shuffle=True)
    set_epoch((dl, plain), 0)
    e0 = list(iter(s))
    set_epoch((dl, plain), 1)
    e1 = list(iter(s))
    assert s.epoch == 1 and sorted(e0) != e0 and e0 != e1


def test_discriminator_state_dict_matches_reference():
    """models/vocoder/HiFiGAN.Discriminator builds its parameters exactly as the
    reference (same modules, init order and weight_norm): the seeded state_dict
    equals the reference's (tests/golden/discriminator.npz, seed 93) bit for bit,
    keys included (weight_g / weight_v on the MPD convs, plain weights on the MSD)."""
    import warnings
    from conftest import golden
    from test_gpu_gan import D_PARAMS
    from models.vocoder.HiFiGAN import Discriminator
    g = golden("discriminator")
    torch.manual_seed(93)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        D = Discriminator(**D_PARAMS)
    sd = D.state_dict()
    ref = {k[3:]: v for k, v in g.items() if k.startswith("sd.")}
    assert list(sd) == list(ref)
    for k, v in sd.items():
        assert torch.equal(v, torch.from_numpy(ref[k])), k


def test_dconv_geometry_matches_torch_conv_lengths():
    """Phase-view tap geometry (sel_dconv_geometry) covers exactly the taps of a
    strided, symmetrically padded torch conv."""
    from sel import dconvops as DC
    for Kt, s, pad in ((41, 4, 20), (41, 2, 20), (41, 1, 20), (5, 3, 2), (15, 1, 7), (2, 1, 1), (3, 1, 1)):
        K, q0 = DC.geometry(Kt, s, pad)
        taps = [s * (q0 + i) + r + pad for i in range(K) for r in range(s)]
        # every torch tap k is exactly one phase-view (i, r); the others are structural zeros
        assert sorted(k for k in taps if 0 <= k < Kt) == list(range(Kt))
        # and no phase-view tap is entirely padding (K is minimal)
        assert any(0 <= s * q0 + r + pad < Kt for r in range(s))
        assert any(0 <= s * (q0 + K - 1) + r + pad < Kt for r in range(s))


def test_c5_mpd_layers_take_the_flat_warp_specialised_tiles():
    """The launcher's own decision (sel_dconv_kernel, no GPU needed) for the MPD
    chain at C5 sizes in the period_alloc layout: the wide layers (1-4 forward,
    2-4 adjoint) run on k_conv_ws_bf16 with flat tiles across sequences
    (SEL_DPATH_WS_FLAT), which tests/test_gpu_c5.py checks numerically; tune
    key 22 = 1 moves them to per-sequence tiles."""
    import ctypes
    from oracle import ref_ops as R
    from sel import _lib as L
    from sel import dconvops as DC
    specs = [DC.LayerSpec(ci, co, k, s, p, 1, lk) for (ci, co, k, s, p, lk) in R.period_discriminator_plan()]
    lib = L.load()
    for clips in (16, 32):
        for p in (2, 3, 5, 7, 11):
            Lv, Bs = (48000 + p - 1) // p, clips * p
            geo = DC.chain_layout(specs, Lv, DC.period_alloc(Lv, specs))
            fwd, adj = [], []
            for li, (sp, (Ti, Ta, To, Toa)) in enumerate(zip(specs, geo)):
                fwd.append(DC.kernel(DC._fwd_desc(sp, Bs, Ti, Ta, To, Toa, 0.1), torch.bfloat16))
                adj.append(DC.kernel(DC._dgrad_desc(sp, Bs, Ta, To, Toa, 0.1, li > 0, T_in=Ti), torch.bfloat16))
            assert [f[0] for f in fwd[1:5]] == ["ws_flat"] * 4, (clips, p, fwd)
            assert [a[0] for a in adj[2:5]] == ["ws_flat"] * 3, (clips, p, adj)
            # the 128 -> 512 layer on the eight-wave 256 x 256 kernel, the others on the 12-wave one
            assert fwd[4][1] == "k_conv_ws_bf16<5>" and fwd[1][1] == "k_conv_ws_bf16<2>"
            assert fwd[3][1] == "k_conv_ws_bf16<2>" and fwd[2][1] == "k_conv_ws8<2, bf16, 256, 256>"
            prev = lib.sel_tune(37, 1)
            try:
                assert DC.kernel(DC._fwd_desc(specs[2], Bs, *geo[2], 0.1), torch.bfloat16)[1] == "k_conv_ws_bf16<2>"
            finally:
                lib.sel_tune(37, prev)
            prev = lib.sel_tune(22, 1)
            try:
                d = DC._fwd_desc(specs[2], Bs, *geo[2], 0.1)
                assert DC.kernel(d, torch.bfloat16)[0] == "ws"
            finally:
                lib.sel_tune(22, prev)
    # invalid descriptors are reported, not guessed
    assert lib.sel_dconv_kernel(ctypes.byref(DC.DConvDesc()), 1, None, 0) == -1


def test_trainer_checkpoint_roundtrip_with_reference_file(tmp_path):
    """TrainerGAN.save_checkpoint / load_checkpoint (trainerGAN.py:95-149): our
    trainer loads the checkpoint the REFERENCE trainer saved
    (tests/golden/trainer_ckpt.pt: reduced PQC generator + HiFi-GAN discriminator,
    Adam / StepLR / MultiStepLR states), with load_only_params both ways, and
    writes back a dict of the identical structure and values."""
    import warnings
    from conftest import GOLDEN
    from test_gpu_gan import D_PARAMS
    from models.autoencoder.AudioDec import Generator
    from models.vocoder.HiFiGAN import Discriminator
    from trainer.denoise import Trainer
    ref_path = os.path.join(GOLDEN, "trainer_ckpt.pt")
    ref = torch.load(ref_path, map_location="cpu", weights_only=True)
    gp = dict(encode_channels=4, decode_channels=4, code_dim=64, codebook_num=2, codebook_size=64)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        G, D = Generator(**gp), Discriminator(**D_PARAMS)
    og = torch.optim.Adam(G.parameters(), lr=1e-4, betas=(0.5, 0.9))
    od = torch.optim.Adam(D.parameters(), lr=2e-4, betas=(0.5, 0.9))
    tr = Trainer(steps=0, epochs=0, data_loader={}, model={"generator": G, "discriminator": D}, criterion={},
                 optimizer={"generator": og, "discriminator": od},
                 scheduler={"generator": torch.optim.lr_scheduler.StepLR(og, 200000, 1.0),
                            "discriminator": torch.optim.lr_scheduler.MultiStepLR(od, [200000, 400000], 0.5)},
                 config={"outdir": None})
    tr.load_checkpoint(ref_path, load_only_params=True)
    assert tr.steps == 0
    for k, v in ref["model"]["generator"].items():
        assert torch.equal(G.state_dict()[k], v), k
    tr.load_checkpoint(ref_path)
    assert tr.steps == ref["steps"] == 2 and tr.epochs == ref["epochs"]
    out = tmp_path / "ck" / "checkpoint-2steps.pkl"
    tr.save_checkpoint(str(out))
    mine = torch.load(out, map_location="cpu", weights_only=True)

    def same(a, b, path=""):
        assert type(a) == type(b) or (isinstance(a, (list, tuple)) and isinstance(b, (list, tuple))), path
        if isinstance(a, dict):
            assert list(a) == list(b), (path, set(a) ^ set(b))
            for k in a:
                same(a[k], b[k], f"{path}/{k}")
        elif isinstance(a, (list, tuple)):
            assert len(a) == len(b), path
            for i, (x, y) in enumerate(zip(a, b)):
                same(x, y, f"{path}[{i}]")
        elif torch.is_tensor(a):
            assert torch.equal(a, b), path
        else:
            assert a == b, path
    same(mine, ref)


def test_rvq_codebook_stack_cache_follows_updates():
    """ResidualVQ._stacked: the (S, D, K) codebook stack is reused while no
    codebook changes and rebuilt after an in-place update (EMA / load_state_dict)."""
    from layers.vq_module import ResidualVQ
    torch.manual_seed(0)
    rvq = ResidualVQ(num_quantizers=3, dim=8, codebook_size=16)
    a = rvq._stacked()
    assert rvq._stacked() is a
    assert torch.equal(a, torch.stack([l.embed for l in rvq.layers]))
    with torch.no_grad():
        rvq.layers[1].embed.mul_(2.0)
    b = rvq._stacked()
    assert b is not a and torch.equal(b, torch.stack([l.embed for l in rvq.layers]))
    sd = {k: v.clone() + 1.0 for k, v in rvq.state_dict().items()}
    rvq.load_state_dict(sd)
    assert torch.equal(rvq._stacked(), torch.stack([l.embed for l in rvq.layers]))
    # a write through .data bumps no version: invalidate_codebook() is the contract
    c = rvq._stacked()
    rvq.layers[2].embed.data.add_(1.0)
    assert rvq._stacked() is c
    rvq.layers[2].invalidate_codebook()
    assert torch.equal(rvq._stacked(), torch.stack([l.embed for l in rvq.layers]))
    # load_state_dict of the same values into the same storage still rebuilds
    d = rvq._stacked()
    rvq.load_state_dict({k: v.clone() for k, v in rvq.state_dict().items()})
    assert rvq._stacked() is not d
