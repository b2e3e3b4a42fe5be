"""bench.py's own multi-rank path, executed: `torch.distributed.run
--nproc-per-node 2 bench.py --gpus 2` as the driver launches it for the
scaling runs, on the box's one GPU (both ranks on cuda:0 over gloo: RCCL
cannot place two ranks on one device; SEL_BENCH_BACKEND / SEL_BENCH_SHARE_GPU
are rehearsal knobs, the driver's runs use RCCL with one rank per GPU).

Covers what only the N > 1 bench runs: the DDP-wrapped generator with the
frozen quantizer / decoder, the batch-global add_noise exchange, the
barrier + max-over-ranks step timing, the rank-0 JSON line (n_gpus, weak
scaling, whole-job value), for C3 and for C5 (GAN step with both modules
DDP-wrapped and the concurrent sub-discriminator chains).  The launcher is a
child process; the pytest process never execs."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("cfg", ["c3", "c5"])
def test_bench_two_ranks(cfg, tmp_path):
    env = dict(os.environ, SEL_BENCH_BACKEND="gloo", SEL_BENCH_SHARE_GPU="1",
               HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(REPO, "bench.py"),
           "--gpus", "2", "--config", cfg, "--steps", "2", "--warmup", "1", "--batch", "4",
           "--no-cpu-baseline", "--no-fp32-companion"]
    log = tmp_path / "bench.log"
    with open(log, "w") as f:
        rc = subprocess.call(cmd, cwd=REPO, env=env, stdout=f, stderr=subprocess.STDOUT, timeout=280)
    text = log.read_text()
    assert rc == 0, text[-3000:]
    lines = [ln for ln in text.splitlines() if ln.startswith("{") and '"metric"' in ln]
    assert len(lines) == 1, text[-3000:]  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "weak" and d["value"] > 0, d
    assert d["config"]["global_batch"] == 8 and d["config"]["parallelism"] == "dp2", d["config"]
