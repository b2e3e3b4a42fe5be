"""GPU parity of streaming inference: StreamGenerator
(models/autoencoder/AudioDec.py:106-191) with every causal layer carrying its
pad_buffer (layers/conv_layer.py:144-191), against the reference-generated
golden (tests/golden/stream.npz, reduced width) and, at full width, against the
oracle restatement (oracle/ref_ops.py stream_*), which tests/test_oracle_goldens.py
pins to the same golden.  fp32: <= 1e-5 norm-wise per chunk; VQ indices exact.
Also: chunked streaming of the conv stack equals one-shot forward on the whole
signal wherever the reference's semantics make them equal (zero initial state,
stride-aligned chunks: the causal convs; the transposed convs differ only in
the first s samples, where forward replicates and streaming starts from zero)."""
import numpy as np
import pytest
import torch

from conftest import golden

pytestmark = pytest.mark.gpu

GP = dict(encode_channels=4, decode_channels=4, code_dim=64, codebook_num=2, codebook_size=64)


def nclose(a, b, rtol, name=""):
    a, b = (v.detach().float().cpu().numpy().astype(np.float64) if torch.is_tensor(v) else np.asarray(v, np.float64)
            for v in (a, b))
    assert a.shape == b.shape, (name, a.shape, b.shape)
    e = np.linalg.norm(a - b) / (np.linalg.norm(b) + 1e-30)
    assert e <= rtol, (name, e)


def _stream_model(gpu, g=None, **gp):
    from models.autoencoder.AudioDec import StreamGenerator
    torch.manual_seed(93)
    G = StreamGenerator(**(gp or GP))
    if g is not None:
        G.load_state_dict({k[3:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("sd.")}, strict=True)
    return G.to(gpu).eval()


def test_stream_generator_matches_reference_golden(gpu):
    g = golden("stream")
    G = _stream_model(gpu, g)
    zq0 = G.initial_encoder(600, gpu)
    nclose(zq0, g["init.zq"], 1e-5, "init.zq")
    G.initial_decoder(zq0)
    x = torch.from_numpy(g["x"]).to(gpu)
    for c in range(6):
        z = G.encode(x[:, :, 600 * c:600 * (c + 1)])
        nclose(z, g[f"z.{c}"], 1e-5, f"z.{c}")
        idx = G.quantize(z)
        np.testing.assert_array_equal(idx.cpu().numpy(), g[f"idx.{c}"])
        zq = G.lookup(idx)
        nclose(zq, g[f"zq.{c}"], 1e-5, f"zq.{c}")
        nclose(G.decode(zq), g[f"y.{c}"], 1e-5, f"y.{c}")
    sd = G.state_dict()
    for k, v in g.items():
        if k.startswith("buf."):
            nclose(sd[k[4:]], v, 1e-5, k)
    G.reset_buffer()
    assert all(float(v.abs().sum()) == 0.0 for k, v in G.state_dict().items() if k.endswith("pad_buffer"))


def test_stream_full_width_vs_oracle(gpu):
    """Full-width AudioDec (32 channels, 8 x 1024 codes): 4 chunks of 1200 samples."""
    from oracle import ref_ops as R
    G = _stream_model(gpu, None, encode_channels=32, decode_channels=32, code_dim=64, codebook_num=8,
                      codebook_size=1024)
    P = {k: v.detach().cpu() for k, v in G.state_dict().items()}
    geo = R.generator_geometry()
    embeds = [P[f"quantizer.codebook.layers.{i}.embed"] for i in range(8)]
    G.quantizer.initial()
    S = {}
    x = 0.1 * torch.randn(1, 1, 4800, generator=torch.Generator().manual_seed(5))
    for c in range(4):
        xc = x[:, :, 1200 * c:1200 * (c + 1)]
        z = G.encode(xc.to(gpu))
        zr = R.stream_encode(P, S, xc, geo)
        nclose(z, zr, 1e-5, f"z.{c}")
        idx = G.quantize(z)
        ir = R.stream_quantize(zr, embeds)
        # indices: exact unless the two paths' fp32 distances tie at the last ulp
        agree = float((idx.cpu() == ir).float().mean())
        assert agree >= 0.99, agree
        zq = G.lookup(ir.to(gpu))
        nclose(zq, R.stream_lookup(ir, embeds), 1e-6, f"zq.{c}")
        nclose(G.decode(zq), R.stream_decode(P, S, R.stream_lookup(ir, embeds), geo), 1e-5, f"y.{c}")


def test_stream_encoder_chunks_equal_one_shot(gpu):
    """Zero initial state + stride-aligned chunks: streaming the encoder equals its
    one-shot causal forward (the causal convs' zero pad is the zero pad_buffer)."""
    G = _stream_model(gpu, None, encode_channels=8, decode_channels=8, code_dim=64, codebook_num=2,
                      codebook_size=64)
    x = 0.1 * torch.randn(1, 1, 6000, generator=torch.Generator().manual_seed(7)).to(gpu)
    with torch.no_grad():
        z_full = G.projector(G.encoder(x))
    G.reset_buffer()
    z_chunks = torch.cat([G.encode(x[:, :, 1200 * c:1200 * (c + 1)]) for c in range(5)], -1)
    nclose(z_chunks, z_full, 1e-5, "z")


def test_stream_without_pqc_chunks_vs_oracle(gpu):
    """without_PQC StreamGenerator: encoder.encode -> decoder.decode (conv1 skipped)."""
    from oracle import ref_ops as R
    from models.autoencoder_without_PQC.AudioDec import StreamGenerator
    torch.manual_seed(3)
    G = StreamGenerator(encode_channels=8, decode_channels=8, code_dim=64, codebook_num=2,
                        codebook_size=64).to(gpu).eval()
    P = {k: v.detach().cpu() for k, v in G.state_dict().items()}
    geo = R.generator_geometry(encode_channels=8, decode_channels=8)
    S = {}
    x = 0.1 * torch.randn(1, 1, 3600, generator=torch.Generator().manual_seed(9))
    for c in range(3):
        xc = x[:, :, 1200 * c:1200 * (c + 1)]
        h = G.encode(xc.to(gpu))
        S_enc = R.stream_encode(P, S, xc, geo, project=False)
        nclose(h, S_enc, 1e-5, f"h.{c}")
        nclose(G.decode(h), R.stream_decode(P, S, S_enc.transpose(2, 1), geo, pqc=False), 1e-5, f"y.{c}")


def test_kernel1_causal_conv_inference_keeps_whole_input(gpu):
    """A kernel-1 CausalConv1d streams as the reference's inference does
    (conv_layer.py:144-147 with pad_length 0): the buffer becomes the whole
    concatenated input (x[:, :, -0:]), so the second call returns the conv over
    both chunks."""
    from layers.conv_layer import CausalConv1d
    torch.manual_seed(3)
    conv = CausalConv1d(16, 24, kernel_size=1).to(gpu).eval()
    x1 = torch.randn(1, 16, 40, device=gpu)
    x2 = torch.randn(1, 16, 24, device=gpu)
    with torch.no_grad():
        y1 = conv.inference(x1)
        y2 = conv.inference(x2)
        w, b = conv.conv.weight.cpu(), conv.conv.bias.cpu()   # reference on the host
        ref1 = torch.nn.functional.conv1d(x1.cpu(), w, b)
        ref2 = torch.nn.functional.conv1d(torch.cat((x1, x2), -1).cpu(), w, b)
    assert conv.pad_buffer.shape == (1, 16, 64)
    nclose(y1, ref1, 1e-5, "y1")
    nclose(y2, ref2, 1e-5, "y2")
