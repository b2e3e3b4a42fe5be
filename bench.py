"""Benchmark of the denoise-training hot path on MI355X.

python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c2]
(N > 1: launched by torch.distributed.run, one rank per GPU over RCCL.)

Prints ONE JSON line (rank 0): BASELINE.json's metric "denoise-train frames/sec
(24 kHz, hop 300)" — frames = clips x 24000 / 300 — for the whole job, with
a live `roofline` for the dominant kernel (HIP events on its launch stream) and
a `cpu_baseline` (the oracle, timed on this host's cores on a bounded sample).

Workloads (BASELINE.json configs):
  c3 (default): configs[2] — one full denoise-trainer step (trainer/denoise.py):
      PQC generator fwd/bwd (decoder + quantizer frozen, codebook eval),
      45 x mel loss + vq loss, clip, Adam; B = 64 x 1 s @ 24 kHz per GPU.
  c2: configs[1] — spectral losses only (3-res STFT + 24 kHz mel), fwd+bwd, B=32, fp32.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "dl-speech-enhancement_amd")
for _p in (REPO, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

SR = 24000
HOP = 300
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
MEL24 = dict(fs=24000, fft_sizes=[2048], hop_sizes=[300], win_lengths=[None], window="hann_window",
             num_mels=80, fmin=0, fmax=24000, log_base=None)
STFT_RES = [(1024, 120, 600), (2048, 240, 1200), (512, 50, 240)]


def synthetic_batch(B, T, seed=93):
    """clean = 0.1*N(0,1) (PCG64(93)), noise PCG64(94), mixed = add_noise(snr=15)."""
    clean = (0.1 * np.random.Generator(np.random.PCG64(seed)).standard_normal((B, 1, T))).astype(np.float32)
    noise = (0.1 * np.random.Generator(np.random.PCG64(seed + 1)).standard_normal((B, 1, T))).astype(np.float32)
    return torch.from_numpy(clean), torch.from_numpy(noise)


def _median_time(step, steps):
    ts = []
    for _ in range(steps):
        t0 = time.perf_counter()
        step()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts))


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown CPU"


# ---------------------------------------------------------------------------
# c2: spectral losses only
# ---------------------------------------------------------------------------

def c2_setup(dev, B):
    from losses import MultiMelSpectrogramLoss, MultiResolutionSTFTLoss
    clean, noise = synthetic_batch(B, SR)
    y_hat = (clean + 0.3 * noise).to(dev)
    y = clean.to(dev)
    mel = MultiMelSpectrogramLoss(**MEL24).to(dev)
    stft = MultiResolutionSTFTLoss().to(dev)
    x = y_hat.clone().requires_grad_(True)

    def step():
        x.grad = None
        sc, mg = stft(x, y)
        loss = 45.0 * mel(x, y) + 45.0 * (sc + mg)
        loss.backward()
    return step


def c2_cpu_baseline(B_sample=4, steps=20):
    from oracle import ref_ops as R
    from oracle.melfilters import mel as melbank
    mm = torch.from_numpy(melbank(sr=24000, n_fft=2048, n_mels=80, fmin=0, fmax=24000).T.copy())
    clean, noise = synthetic_batch(B_sample, SR)
    y = clean
    x = (clean + 0.3 * noise).requires_grad_(True)
    wins = [R.hann(w) for _, _, w in STFT_RES]

    def step():
        x.grad = None
        sc, mg = R.mr_stft_loss(x, y, STFT_RES, wins)
        loss = 45.0 * R.multi_mel_loss(x, y, [(2048, 300, 2048)], [R.hann(2048)], [mm], 1e-10, None) \
            + 45.0 * (sc + mg)
        loss.backward()
    step()
    dt = _median_time(step, steps)
    return B_sample * SR / HOP / dt, (f"oracle (PyTorch-CPU restatement) c2 losses fwd+bwd, B={B_sample}, "
                                      f"median of {steps} steps, on {_cpu_model()}")


# ---------------------------------------------------------------------------
# c3: full denoise-trainer step
# ---------------------------------------------------------------------------

C3_CONFIG = "symAD_libritts_24000_hop300"


# rehearsal knob (not a driver configuration): SEL_BENCH_FORCE_DDP=1 runs the
# N = 1 step DDP-wrapped under a one-rank process group, i.e. the data-parallel
# schedule (bucket copies, the sel comm hook's per-bucket weight-gradient
# reductions, the all-reduce calls) without the interconnect
FORCE_DDP = os.environ.get("SEL_BENCH_FORCE_DDP", "0") == "1"


def c3_setup(dev, B, world, local, graph=False, dtype=torch.bfloat16, batch=None):
    """The timed C3 step.  batch: an explicit GLOBAL (clean, noise) pair of CPU
    tensors instead of the synthetic per-rank one (each rank takes its shard):
    tests/ddp_product_worker.py's "bench" case runs this very step under a
    process group against one process on the same global batch."""
    from sel import configs
    from sel.convops import precision
    from models.autoencoder.AudioDec import Generator
    from losses import MultiMelSpectrogramLoss
    from trainer.denoise import Trainer
    from dataloader.data_utils import add_noise

    cfg = configs.get(C3_CONFIG)
    cfg["outdir"] = None
    cfg["train_max_steps"] = 1 << 40
    torch.manual_seed(93)
    G = Generator(**cfg["generator_params"]).to(dev)
    model = {"generator": G, "discriminator": None}
    if world > 1 or FORCE_DDP:
        from sel.dist import wrap_ddp
        # freeze first so DDP only buckets the trainable (encoder + projector) grads
        for p in list(G.quantizer.parameters()) + list(G.decoder.parameters()):
            p.requires_grad = False
        # sel.ddp: 4 MB buckets, the deferred weight-gradient reductions per bucket
        model["generator"] = wrap_ddp(G, dev, force=FORCE_DDP)
    mel = MultiMelSpectrogramLoss(**cfg["mel_loss_params"]).to(dev)
    opt_kw = dict(cfg["generator_optimizer_params"])
    if graph:
        opt_kw["capturable"] = True  # step count and lr on device: the update replays inside a HIP graph
    if os.environ.get("SEL_ADAM_FOREACH", "0") != "1":
        # one fused multi-tensor Adam launch instead of torch's 7 foreach passes
        # (128 us/step at C3, profiles/r1_c3_v22_kernel_stats.md); same update rule
        opt_kw.setdefault("fused", True)
    # sel.optim.Adam (one sel_adam_step_many launch; capturable: the device-count
    # form sel_adam_step_many_dev) unless SEL_ADAM=torch
    from sel import optim as sel_optim
    opt = sel_optim.adam(G.parameters(), **opt_kw)
    sched = torch.optim.lr_scheduler.StepLR(opt, **cfg["generator_scheduler_params"])
    tr = Trainer(steps=0, epochs=0, data_loader={}, model=model, criterion={"mel": mel},
                 optimizer={"generator": opt}, scheduler={"generator": sched}, config=cfg, device=dev)
    if batch is None:
        clean, noise = synthetic_batch(B, SR, seed=93 + 2 * int(os.environ.get("RANK", "0")))
    else:
        from sel.dist import shard
        clean, noise = batch
        if world > 1:
            clean, noise = shard(clean), shard(noise)
    clean, noise = clean.to(dev), noise.to(dev)
    if world > 1:
        # batch-global add_noise norms over all ranks' shards (data_utils.py:15-16)
        from sel.dist import add_noise_global
        mixed = add_noise_global(clean, noise, 15)
    else:
        mixed = add_noise(clean, noise, 15)

    def step():
        with precision(dtype):
            tr._train_step((mixed, clean))
    if graph:
        # the whole trainer step as one HIP-graph replay (trainer/graph.py)
        from trainer.graph import GraphedTrainStep
        with precision(dtype):
            gs = GraphedTrainStep(tr, (mixed, clean))
        gs.eager = step
        gs.trainer, gs.generator = tr, G
        return gs
    step.trainer, step.generator = tr, G
    return step


def c3_cpu_baseline(B_sample=4, steps=20):
    """Oracle (op-for-op PyTorch-CPU restatement) of the same denoise-trainer step."""
    from oracle import ref_ops as R
    from oracle.melfilters import mel as melbank
    from sel import configs
    cfg = configs.get(C3_CONFIG)
    mp = cfg["mel_loss_params"]
    mm = torch.from_numpy(melbank(sr=mp["fs"], n_fft=2048, n_mels=80, fmin=mp["fmin"], fmax=mp["fmax"]).T.copy())
    torch.manual_seed(93)
    from models.autoencoder.AudioDec import Generator
    P = {k: v.clone() for k, v in Generator(**cfg["generator_params"]).state_dict().items()}
    train = [k for k in P if (k.startswith("encoder.") or k.startswith("projector.")) and
             (k.endswith("weight") or k.endswith("bias"))]
    for k in train:
        P[k].requires_grad_(True)
    opt = torch.optim.Adam([P[k] for k in train], **cfg["generator_optimizer_params"])
    geo = R.generator_geometry()
    clean, noise = synthetic_batch(B_sample, SR)
    mixed = R.add_noise(clean, noise, 15)
    win = R.hann(2048)

    def step():
        y, zq, z, vql, ppl = R.generator_forward(P, mixed, geo, pqc=True)
        loss = vql.sum() * cfg["lambda_vq_loss"] + cfg["lambda_mel_loss"] * R.multi_mel_loss(
            y, clean, [(2048, 300, 2048)], [win], [mm], 1e-10, None)
        opt.zero_grad()
        loss.backward()
        opt.step()
    step()
    dt = _median_time(step, steps)
    return B_sample * SR / HOP / dt, (f"oracle (PyTorch-CPU op-for-op restatement) denoise-trainer step, "
                                      f"PQC generator fp32, B={B_sample} x 1 s, median of {steps} timed steps "
                                      f"after 1 warm-up, on {_cpu_model()}")


C1_CONFIG = "symAD_24Mel"


def c1_cpu_baseline(B=2, steps=5):
    """BASELINE configs[0] as named: the reference's CPU case — train_denoise.py's
    default symAD_24Mel step (without-PQC generator, 45 x mel + 0 x SNR, clip
    norm 1, Adam; :213-263 before the discriminator is enabled) at B = 2 x 1 s @
    24 kHz, on the oracle's op-for-op restatement."""
    from oracle import ref_ops as R
    from oracle.melfilters import mel as melbank
    from sel import configs
    from models.autoencoder_without_PQC.AudioDec import Generator
    cfg = configs.get(C1_CONFIG)
    mp = cfg["mel_loss_params"]
    mm = torch.from_numpy(melbank(sr=mp["fs"], n_fft=2048, n_mels=80, fmin=mp["fmin"], fmax=mp["fmax"]).T.copy())
    torch.manual_seed(93)
    P = {k: v.clone() for k, v in Generator(**cfg["generator_params"]).state_dict().items()}
    train = [k for k in P if k.startswith(("encoder.", "decoder.conv_blocks", "decoder.conv2"))
             and not k.endswith("pad_buffer")]
    for k in train:
        P[k].requires_grad_(True)
    params = [P[k] for k in train]
    opt = torch.optim.Adam(params, **cfg["generator_optimizer_params"])
    geo = R.generator_geometry(**cfg["generator_params"])
    clean, noise = synthetic_batch(B, SR)
    mixed = R.add_noise(clean, noise, 15)
    win = R.hann(2048)

    def step():
        y = R.generator_forward(P, mixed, geo, pqc=False)
        loss = cfg["lambda_mel_loss"] * R.multi_mel_loss(y, clean, [(2048, 300, 2048)], [win], [mm], 1e-10, None)
        opt.zero_grad()
        loss.backward()
        torch.nn.utils.clip_grad_norm_(params, cfg["generator_grad_norm"])
        opt.step()
    step()
    dt = _median_time(step, steps)
    return {"value": round(B * SR / HOP / dt, 1), "unit": "frames/s", "ms_per_step": round(dt * 1e3, 1),
            "sample": (f"configs[0] as named: {C1_CONFIG} train_denoise step (without-PQC generator, mel, clip, "
                       f"Adam), B={B} x 1 s @ 24 kHz, fp32 oracle, median of {steps} steps after 1 warm-up, on "
                       f"{_cpu_model()}")}


# ---------------------------------------------------------------------------
# c5: GAN-mode denoise step at 48 kHz (generator + HiFi-GAN MSD/MPD discriminator)
# ---------------------------------------------------------------------------

C5_CONFIG = "symAD_vctk_48000_hop300"
SR48 = 48000


def c5_setup(dev, B, world, local, dtype=torch.bfloat16):
    """train_denoise.py model_step in GAN mode (:138-165, :213-263): generator
    45*mel + adv + 2*feat-match, Adam; discriminator real/fake LSGAN, Adam."""
    from sel import configs
    from sel.convops import precision
    from models.autoencoder_without_PQC.AudioDec import Generator
    from models.vocoder.HiFiGAN import Discriminator
    from train_denoise import DenoiseStep
    from dataloader.data_utils import add_noise
    cfg = configs.get(C5_CONFIG)
    torch.manual_seed(93)
    G = Generator(**cfg["generator_params"]).to(dev)
    for mod in (G.projector, G.quantizer, G.decoder.conv1):  # unused by the without-PQC forward
        for p in mod.parameters():
            p.requires_grad_(False)
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        D = Discriminator(**cfg["discriminator_params"]).to(dev)
    st = DenoiseStep(cfg, dev, generator=G, discriminator=D)
    if world > 1:
        from sel.dist import wrap_ddp
        st.model["generator"] = wrap_ddp(G, dev)
        st.model["discriminator"] = wrap_ddp(D, dev)
    st.discriminator_enabled = True
    clean, noise = synthetic_batch(B, SR48, seed=93 + 2 * int(os.environ.get("RANK", "0")))
    clean, noise = clean.to(dev), noise.to(dev)
    if world > 1:
        from sel.dist import add_noise_global
        mixed = add_noise_global(clean, noise, 15)
    else:
        mixed = add_noise(clean, noise, 15)

    def step():
        with precision(dtype):
            st.model_step(clean, mixed)
    return step


def c5_cpu_baseline(B_sample=1, steps=5):
    """Oracle (op-for-op PyTorch-CPU restatement) of the same GAN step, fp32."""
    from oracle import ref_ops as R
    from oracle.melfilters import mel as melbank
    from sel import configs
    from models.autoencoder_without_PQC.AudioDec import Generator
    from models.vocoder.HiFiGAN import Discriminator
    import warnings
    cfg = configs.get(C5_CONFIG)
    mp = cfg["mel_loss_params"]
    mm = torch.from_numpy(melbank(sr=mp["fs"], n_fft=2048, n_mels=80, fmin=mp["fmin"], fmax=mp["fmax"]).T.copy())
    torch.manual_seed(93)
    Gp = {k: v.clone() for k, v in Generator(**cfg["generator_params"]).state_dict().items()}
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        Dp = {k: v.clone() for k, v in Discriminator(**cfg["discriminator_params"]).state_dict().items()}
    gtrain = [k for k in Gp if k.startswith(("encoder.", "decoder.conv_blocks", "decoder.conv2"))
              and not k.endswith("pad_buffer")]
    for k in gtrain:
        Gp[k].requires_grad_(True)
    for v in Dp.values():
        v.requires_grad_(True)
    og = torch.optim.Adam([Gp[k] for k in gtrain], **cfg["generator_optimizer_params"])
    od = torch.optim.Adam(list(Dp.values()), **cfg["discriminator_optimizer_params"])
    dkw = cfg["discriminator_params"]
    geo = R.generator_geometry()
    clean, noise = synthetic_batch(B_sample, SR48)
    mixed = R.add_noise(clean, noise, 15)
    win = R.hann(2048)

    def step():
        pred = R.generator_forward(Gp, mixed, geo, pqc=False)
        mel = R.multi_mel_loss(pred, clean, [(2048, 300, 2048)], [win], [mm], 1e-10, None)
        p_ = R.hifigan_discriminator(Dp, pred, **dkw)
        with torch.no_grad():
            p = R.hifigan_discriminator(Dp, clean, **dkw)
        gen = cfg["lambda_mel_loss"] * mel + cfg["lambda_adv"] * R.generator_adv_loss(pred, False) + \
            cfg["lambda_feat_match"] * R.feat_match_loss(p_, p)
        og.zero_grad()
        gen.backward()
        og.step()
        with torch.no_grad():
            pred2 = R.generator_forward(Gp, mixed, geo, pqc=False)
        rl, fl = R.discriminator_adv_loss(R.hifigan_discriminator(Dp, pred2, **dkw),
                                          R.hifigan_discriminator(Dp, clean, **dkw), False)
        od.zero_grad()
        (rl + fl).backward()
        od.step()
    step()
    dt = _median_time(step, steps)
    return B_sample * SR48 / HOP / dt, (f"oracle (PyTorch-CPU op-for-op restatement) GAN-mode denoise step, "
                                        f"without-PQC generator + HiFi-GAN MSD/MPD fp32, B={B_sample} x 1 s @ 48 kHz, "
                                        f"median of {steps} timed steps after 1 warm-up, on {_cpu_model()}")


# ---------------------------------------------------------------------------

MFMA_BF16_PEAK_TFS = 2500.0  # MI355X dense bf16 (MI355X_MICROARCH.md)
FP32_PEAK_TFS = 157.3        # MI355X fp32 vector (= fp32 MFMA) peak (MI355X_MICROARCH.md)


def pmc_file(cfg):
    """Newest committed PMC traffic table of a config's bench (tools/gpu.sh pmc):
    profiles/r<round>_<cfg>_pmc_traffic[_v<k>].json, highest (round, k) wins."""
    import glob
    import re
    best, key = "", (-1, -1)
    for f in glob.glob(os.path.join(REPO, "profiles", f"r*_{cfg}_pmc_traffic*.json")):
        m = re.match(rf"r(\d+)_{cfg}_pmc_traffic(?:_v(\d+))?\.json$", os.path.basename(f))
        if m and (int(m.group(1)), int(m.group(2) or 0)) > key:
            best, key = f, (int(m.group(1)), int(m.group(2) or 0))
    return best


def _mangled_fragment(tag):
    """'k_conv_fwd_bf16<128, 64, 2, 8, bf16>' -> 'k_conv_fwd_bf16ILi128ELi64ELi2ELi8EDF16b' (Itanium;
    a prefix: a tag may name the leading template arguments only, 'k_conv_ws_bf16<5>')."""
    import re
    m = re.match(r"(\w+)<(.*)>", tag)
    if not m:
        return tag
    parts = []
    for a in (x.strip() for x in m.group(2).split(",")):
        parts.append({"bf16": "DF16b", "float": "f"}.get(a, f"Li{a}E"))
    return m.group(1) + "I" + "".join(parts)


DEFAULT_BATCH = {"c2": 32, "c3": 64, "c5": 16}


def pmc_traffic(tag, B, cfg="c3"):
    """HBM bytes per launch of kernel `tag` from the committed rocprofv3 PMC passes
    (tools/pmc_traffic.py over FETCH_SIZE / WRITE_SIZE runs of this same bench
    command, gfx950 corrections applied there), or None if not measured."""
    path = pmc_file(cfg)
    if B != DEFAULT_BATCH.get(cfg) or not path:
        return None
    frag = _mangled_fragment(tag)
    with open(path) as f:
        table = json.load(f)
    # a tag can cover several compiled variants (e.g. the thin kernel's
    # epilogue-prefetch template flag: ...ELb0E / ...ELb1E): launch-weighted mean
    hits = [v for k, v in table.items() if frag in k or k.split("(")[0].endswith(tag)]
    if not hits:
        return None
    n = sum(v["launches"] for v in hits)
    return int(sum(v["traffic_bytes_per_launch"] * v["launches"] for v in hits) / n)


def roofline(cfg, timer, dom, B, steps):
    """Dominant timed kernel instance -> achieved vs peak (HIP events, same stream)."""
    summ = timer.summary()
    total_ms = sum(v[1] for v in summ.values())
    ranked = sorted(summ.items(), key=lambda kv: kv[1][1], reverse=True)
    # c2 computes in fp32 (the FFTs on the vector ALUs): its compute roof is
    # the fp32 vector peak; c3 / c5 convs run bf16 MFMA
    peak = FP32_PEAK_TFS if cfg == "c2" else MFMA_BF16_PEAK_TFS
    top = [_roof_entry(tag, v, total_ms, B, cfg, peak) for tag, v in ranked[:3]]
    r = dict(top[0])
    r["top3"] = top
    r["timed_entry_points"] = sorted(timer.names)
    return r


# the fused residual-unit forwards also write h = conv1(ELU(x)) for the
# backward: a design choice (the backward could recompute it from x), whose
# bytes are counted in the kernel's algorithmic bytes (one of its three
# activation tensors)
H_STASH = {"k_ru32_fwd", "k_ru64_fwd"}


def _roof_entry(tag, v, total_ms, B, cfg, peak_tfs=None):
    """One timed kernel instance -> achieved vs its roofline (mfma when its
    arithmetic intensity is past the bf16 ridge, else hbm)."""
    n, ms, nbytes, flops = v
    peak_tfs = peak_tfs or MFMA_BF16_PEAK_TFS
    intensity = flops / max(nbytes, 1)
    ridge = peak_tfs * 1e12 / (HBM_PEAK_GBS * 1e9)
    if nbytes == 0 and flops == 0:
        r = {"bound": None, "achieved": None, "peak": None, "unit": None, "frac": None}
    elif intensity > ridge:
        ach = flops / (ms * 1e-3) / 1e12
        r = {"bound": "mfma" if peak_tfs == MFMA_BF16_PEAK_TFS else "valu-fp32", "achieved": round(ach, 1),
             "peak": peak_tfs, "unit": "TFLOP/s", "frac": round(ach / peak_tfs, 4)}
    else:
        ach = nbytes / (ms * 1e-3) / 1e9
        r = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
             "frac": round(ach / HBM_PEAK_GBS, 4)}
    r.update({"kernel": tag, "launches": n, "event_timed_steps": 1, "avg_launch_us": round(1e3 * ms / n, 2),
              "bytes_per_launch": int(nbytes / n), "flops_per_launch": int(flops / n),
              "share_of_timed_ms": round(ms / total_ms, 3),
              "traffic": pmc_traffic(tag, B, cfg), "traffic_unit": "bytes/launch (rocprofv3 PMC, profiles/)",
              "traffic_file": os.path.basename(pmc_file(cfg)) or None})
    if tag.split("<")[0] in H_STASH:
        r["note"] = ("bytes include the h stash (1 of 3 activation tensors; a design choice: "
                     "the backward could recompute h from x)")
    return r


def stft_kernel_roofline(dev, B=2048):
    """North-star STFT target: the |X| kernel (sel_stft_mag_fwd, the a1 row) at
    1024/120/600 on B = 2048 x 1 s (0.2 GB in, 0.85 GB out: a working set 4x the
    256 MB Infinity Cache, so nothing is served from it across launches), timed
    with a HIP event pair around each launch on its stream, against the 8 TB/s
    spec and against two measured copy rates of this box: a float4 stream-copy
    kernel (sel_probe_copy_f4: one 16-B nontemporal load and store per thread,
    one-shot grid, 6.4 TB/s; tools/copy_probe.py sweeps its other forms) and
    torch's copy_, each over 1 GiB buffers."""
    from sel import _lib as L
    T, (n, h, w) = SR, STFT_RES[0]
    F, K = 1 + T // h, n // 2 + 1
    x = 0.1 * torch.randn(B, T, device=dev)
    win = torch.hann_window(w, device=dev)
    mag = torch.empty(B, F, K, device=dev)
    src = torch.empty(2 ** 28, device=dev)
    dst = torch.empty_like(src)
    cus = torch.cuda.get_device_properties(dev).multi_processor_count

    def launches(fn, iters=15):
        """per-launch event-pair times in s (back-to-back Python launches leave
        host gaps between short kernels that one pair around a loop would count)"""
        for _ in range(2):
            fn()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
        for e0, e1 in ev:
            e0.record()
            fn()
            e1.record()
        torch.cuda.synchronize()
        return [e0.elapsed_time(e1) * 1e-3 for e0, e1 in ev]

    def timed(fn):
        """median of 15 launches: the sustained rate.  The |X| kernel slows under
        back-to-back load while the copy probe stays flat (tools/stft_clock_trace.py,
        profiles/r6_stft_launch_trace.txt: ~256 us for the first launches, up to
        ~360 around the tenth, ~305-315 after forty; consistent with a power /
        clock limit on the VALU-heavy FFT), so the round-5 protocol (mean of the
        first five timed launches) is kept beside it as the burst rate."""
        ts = launches(fn)
        return sorted(ts)[len(ts) // 2], sum(ts[:5]) / 5

    copy_bytes = 2 * src.numel() * 4
    t_torch = timed(lambda: dst.copy_(src))[0]
    t_f4 = timed(lambda: L.call("sel_probe_copy_f4", L.ptr(src), L.ptr(dst), src.numel() // 4, 8 * cus, L.stream()))[0]
    torch_gbs, f4_gbs = copy_bytes / t_torch / 1e9, copy_bytes / t_f4 / 1e9
    del src, dst
    t, t_burst = timed(lambda: L.call("sel_stft_mag_fwd", L.ptr(x), B, T, n, h, w, L.ptr(win), 1e-7, L.ptr(mag),
                                      L.stream()))
    nbytes = 4 * B * (T + F * K)
    gbs = nbytes / t / 1e9
    return {"kernel": "k_stft_mag_fwd<10>", "shape": f"B={B} x {T}, n_fft/hop/win {n}/{h}/{w}",
            "median_launch_us": round(t * 1e6, 1), "launches": 15, "alg_bytes": nbytes, "achieved": round(gbs, 1),
            "unit": "GB/s",
            "frac_of_spec": round(gbs / HBM_PEAK_GBS, 4),
            "copy_f4_GBs": round(f4_gbs, 1), "frac_of_copy_f4": round(gbs / f4_gbs, 4),
            "torch_copy_GBs": round(torch_gbs, 1), "frac_of_torch_copy": round(gbs / torch_gbs, 4),
            "burst": {"mean_first5_us": round(t_burst * 1e6, 1),
                      "frac_of_copy_f4": round(nbytes / t_burst / 1e9 / f4_gbs, 4)}}


def launch_cmd(n, port, argv):
    """torch.distributed.run command line for N local ranks of this script."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def _relaunch(n):
    """bench.py --gpus N outside torchrun: start N ranks under
    torch.distributed.run as a CHILD process and exit with its code.  Runs
    before anything initialises the GPU (device_count() does not on ROCm)."""
    import socket
    import subprocess
    have = torch.cuda.device_count()
    if have < n:
        sys.exit(f"bench.py: --gpus {n} but only {have} GPU(s) visible")
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = launch_cmd(n, port, sys.argv[1:])
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    sys.exit(subprocess.call(cmd, env=env))


def _timed_steps(step, steps, world, dev, timer=None):
    """K steps bracketed by barrier + synchronize; per-step HIP events on the
    current stream give the per-step durations (max over ranks per step)."""
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
    t0 = time.perf_counter()
    evs[0].record()
    for i in range(steps):
        # per-launch HIP events only in the last timed step: an event pair around
        # every conv launch of every step costs ~0.6 ms/step (C3) of its own
        if timer is not None and i == steps - 1:
            _lib().TIMER = timer
        step()
        evs[i + 1].record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    _lib().TIMER = None
    per = torch.tensor([evs[i].elapsed_time(evs[i + 1]) for i in range(steps)] + [elapsed * 1e3],
                       dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(per, op=dist.ReduceOp.MAX)
    per = per.cpu().numpy()
    return float(per[-1]) * 1e-3, per[:-1]


def _lib():
    from sel import _lib as L
    return L


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="c3", choices=["c2", "c3", "c5"])
    ap.add_argument("--batch", type=int, default=0, help="per-GPU batch (default: config's)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-fp32-companion", action="store_true")
    ap.add_argument("--eager", action="store_true",
                    help="c3: issue every launch from Python instead of replaying the step's HIP graph")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        _relaunch(args.gpus)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal knobs for the multi-rank path on a box with fewer GPUs than
    # ranks (tests only): SEL_BENCH_BACKEND=gloo, SEL_BENCH_SHARE_GPU=1 (rank r
    # on GPU r mod count); the driver's runs use RCCL, one rank per GPU
    backend = os.environ.get("SEL_BENCH_BACKEND", "nccl")
    if os.environ.get("SEL_BENCH_SHARE_GPU", "0") == "1":
        local = local % torch.cuda.device_count()
    if world > 1 or FORCE_DDP:
        torch.cuda.set_device(local)
        if world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(29500 + os.getpid() % 1000))
            os.environ.setdefault("RANK", "0")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), rank=int(os.environ.get("RANK", "0")),
                                    world_size=world)
        else:
            dist.init_process_group(backend, rank=int(os.environ.get("RANK", "0")), world_size=world)
    dev = torch.device("cuda", local)

    from sel import _lib
    cfg = args.config
    B = args.batch or {"c2": 32, "c3": 64, "c5": 16}[cfg]
    sr = SR48 if cfg == "c5" else SR
    if cfg == "c2":
        step = c2_setup(dev, B)
        dom = "sel_stft_loss_fwd"   # + the backward and the fused mel launch (timer below)
        workload = "configs[1]: MR-STFT(3 res) + mel(2048/300/80) loss fwd+bwd, fp32, 1 s @ 24 kHz"
        dtype = "fp32"
    elif cfg == "c3":
        # one process: the trainer step replays as a HIP graph (trainer/graph.py);
        # under a process group the bucketed all-reduce stays eager
        use_graph = world == 1 and not FORCE_DDP and not args.eager and os.environ.get("SEL_BENCH_GRAPH", "1") != "0"
        step = c3_setup(dev, B, world, local, graph=use_graph)
        dom = "sel_conv_fwd"
        workload = (f"configs[2]/[3]: denoise-trainer step (trainer/denoise.py) on the PQC AudioDec generator, "
                    f"{C3_CONFIG} (derived), bf16 convs / fp32 losses, {B} x 1 s @ 24 kHz per GPU")
        dtype = "bf16"
    else:
        step = c5_setup(dev, B, world, local)
        dom = "sel_conv_fwd"
        workload = (f"configs[4]: GAN-mode denoise step (train_denoise.py model_step, discriminator enabled): "
                    f"without-PQC AudioDec generator + HiFi-GAN MSD/MPD discriminator, {C5_CONFIG}, bf16 convs / "
                    f"fp32 losses, {B} x 1 s @ 48 kHz per GPU")
        dtype = "bf16"

    for _ in range(args.warmup):
        step()
    # every entry point that launches a conv-stack kernel of the step (the
    # dominant kernel is the largest total time over all of them)
    timer = (_lib.KernelTimer([dom] + (["sel_resunit_fwd", "sel_resunit_bwd", "sel_resunit_bwd_wgrad",
                                        "sel_conv_wgrad_partials", "sel_wgrad_finish_many"]
                                       if cfg == "c3" else ["sel_stft_loss_bwd", "sel_mel_l1_fwd_grad"]))
             if cfg != "c5" else None)  # C5: a serialised extra step below
    graphed = cfg == "c3" and hasattr(step, "graph")
    elapsed, per_step = _timed_steps(step, args.steps, world, dev, None if graphed else timer)
    if graphed:
        # per-launch HIP events cannot sit inside a replay: the roofline comes
        # from one eager step of the same trainer after the timed region (the
        # same kernels on the same shapes)
        torch.cuda.synchronize()
        _lib.TIMER = timer
        step.eager()
        torch.cuda.synchronize()
        _lib.TIMER = None

    ms_per_step = 1e3 * elapsed / args.steps
    frames_per_step = world * B * sr / HOP
    value = frames_per_step * args.steps / elapsed
    med_ms = float(np.median(per_step))
    if cfg == "c5":
        # the C5 step runs the 8 sub-discriminator chains on side streams: an
        # event pair around one launch there also spans what the other streams
        # run beside it, so the roofline comes from ONE extra step with the
        # chains serialised (SEL_D_STREAMS=0: same kernels, same bits), after
        # the timed region; each launch's events then bracket that launch alone
        prev = os.environ.get("SEL_D_STREAMS")
        os.environ["SEL_D_STREAMS"] = "0"
        timer = _lib.KernelTimer([dom, "sel_dconv_fwd", "sel_dconv_wgrad_partials", "sel_resunit_fwd",
                                  "sel_resunit_bwd", "sel_conv_wgrad_partials", "sel_wgrad_finish_many"])
        torch.cuda.synchronize()
        _lib.TIMER = timer
        step()
        torch.cuda.synchronize()
        _lib.TIMER = None
        if prev is None:
            del os.environ["SEL_D_STREAMS"]
        else:
            os.environ["SEL_D_STREAMS"] = prev
    roof = roofline(cfg, timer, dom, B, 1)  # the timer covered one step (C3: the last timed one)
    if graphed:
        roof["timing"] = "one eager step after the timed graph replays (same kernels)"
    if cfg == "c5":
        roof["timing"] = "one extra step with the sub-discriminator chains serialised (SEL_D_STREAMS=0)"

    fp32 = None
    if cfg == "c3" and not args.no_fp32_companion:
        # the reference's own arithmetic (fp32 convs on the exact-fp32 MFMA path), same step
        step32 = c3_setup(dev, B, world, local, dtype=torch.float32)
        for _ in range(2):
            step32()
        e32, per32 = _timed_steps(step32, args.steps, world, dev)
        fp32 = {"dtype": "fp32", "value": round(frames_per_step * args.steps / e32, 1), "unit": "frames/s",
                "ms_per_step": round(1e3 * e32 / args.steps, 3),
                "median_ms_per_step": round(float(np.median(per32)), 3)}
        del step32

    stft_roof = stft_kernel_roofline(dev) if world == 1 and cfg != "c5" else None
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        ncores = len(os.sched_getaffinity(0))
        ncores = min(ncores, int(os.environ.get("OMP_NUM_THREADS", ncores)))
        torch.set_num_threads(ncores)
        v, sample = {"c2": c2_cpu_baseline, "c3": c3_cpu_baseline, "c5": c5_cpu_baseline}[cfg]()
        cpu = {"value": round(v, 1), "unit": "frames/s", "cores": ncores, "kind": "port", "sample": sample}
        if cfg == "c3":
            cpu["c1"] = c1_cpu_baseline()

    if rank == 0:
        out = {
            "metric": ("denoise-train frames/sec (24 kHz, hop 300)" if cfg != "c5"
                       else "GAN-mode denoise-train frames/sec (48 kHz, hop 300)"),
            "value": round(value, 1), "unit": "frames/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3),
            "median_ms_per_step": round(med_ms, 3),
            "value_at_median": round(frames_per_step / (med_ms * 1e-3), 1),
            "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": dtype, "data": "synthetic",
            "config": {"workload": workload, "global_batch": world * B, "seq_len": sr,
                       "parallelism": f"dp{world}",
                       "issue": "hip-graph replay" if (cfg == "c3" and hasattr(step, "graph")) else "eager"},
            "roofline": roof, "cpu_baseline": cpu, "fp32_companion": fp32, "stft_kernel": stft_roof,
        }
        print(json.dumps(out), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
