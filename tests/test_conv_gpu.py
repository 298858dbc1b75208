"""GPU parity of the fused convNet decoder (npd_conv_forward) against the reference's convNet.forward
logits (golden) and the float64 numpy oracle.

Tolerance (fp32 MFMA vs PyTorch CPU fp32: same operations, different summation order through 10 conv
layers (dot products of up to 7 x 128 terms), 3 FC layers (up to 32768 terms) and LayerNorm): logits
within 1e-5 absolute (LayerNorm output is O(1), |logit| <= 2.3 on the C5 fixture; sqrt(32768) x 2^-24 x
O(1) ~ 1e-5 bounds the typical accumulated rounding); decisions (sign) identical except where the
reference logit is within 1e-5 of zero.  Measured on MI355X (tools/conv_err_report.py): max |diff| =
4.8e-7 (embed 16, N 64, vs reference), 3.6e-7 (vs oracle), 6.0e-7 (C5: embed 128, N 256).
"""
import argparse

import numpy as np
import pytest
import torch

from conftest import conv_weights_from_seed, golden

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
ATOL = 1e-5


def net_from(sd, embed, N, precision="fp32"):
    from neural_polar_decoder_amd.models import convNet
    cfg = argparse.Namespace(embed_dim=embed, max_len=N, N=N, dont_use_bias=False, dropout=0.0)
    net = convNet(cfg, precision=precision)
    net.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
    return net.eval()


def check(lg, dec, ref_lg):
    err = np.abs(lg - ref_lg).max()
    assert err < ATOL, ("max |logit diff|", float(err))
    sure = np.abs(ref_lg) > ATOL
    assert np.array_equal(dec[sure], np.sign(ref_lg)[sure])


def test_conv_small_golden():
    d = golden("conv_small_64.npz")
    sd = {k[2:]: d[k] for k in d.files if k.startswith("w.")}
    net = net_from(sd, int(d["embed"]), int(d["N"]))
    y = torch.from_numpy(d["y"]).to(DEV)
    lg, dec = net.logits(y)
    check(lg.cpu().numpy(), dec.cpu().numpy(), d["logits"])
    out, m = net.decode(y, None, None, DEV)
    assert out.shape == (y.shape[0], int(d["N"]), 1)


def test_conv_c5_golden():
    """C5 shape: embed 128, N = 256 (34.3 M parameters regenerated from the documented seed)."""
    d = golden("conv_c5_256.npz")
    sd = conv_weights_from_seed(int(d["embed"]), int(d["N"]), int(d["seed"]))
    net = net_from(sd, int(d["embed"]), int(d["N"]))
    lg, dec = net.logits(torch.from_numpy(d["y"]).to(DEV))
    check(lg.cpu().numpy(), dec.cpu().numpy(), d["logits"])


def test_conv_vs_oracle_ragged_batch(oracle):
    d = golden("conv_small_64.npz")
    sd = {k[2:]: d[k] for k in d.files if k.startswith("w.")}
    net = net_from(sd, int(d["embed"]), int(d["N"]))
    rng = np.random.default_rng(1)
    y = rng.standard_normal((8192 + 77, 64)).astype(np.float32)  # > one chunk, ragged tail
    lg, dec = net.logits(torch.from_numpy(y).to(DEV))
    ref = oracle.conv_forward(y[::37], sd)
    check(lg.cpu().numpy()[::37], dec.cpu().numpy()[::37], ref)


def test_conv_forward_returns_input4(oracle):
    """convNet.forward's fifth output, input4 = layers3(input3) + input3 (models.py:750, :767), (B, embed/2, N):
    against the reference's value (golden) and the float64 oracle, same 1e-5 bar as the logits (O(1) GELU
    activations, dot products of <= 7 x 64 terms); the other outputs as decode/logits give them."""
    d = golden("conv_small_64.npz")
    sd = {k[2:]: d[k] for k in d.files if k.startswith("w.")}
    net = net_from(sd, int(d["embed"]), int(d["N"]))
    y = torch.from_numpy(d["y"]).to(DEV)
    out, dec, m, logits, in4 = net.forward(y, None, None, DEV)
    assert in4.shape == d["input4"].shape and in4.is_cuda
    assert np.abs(in4.cpu().numpy() - d["input4"]).max() < ATOL
    _, o4 = oracle.conv_forward(d["y"], sd, want_input4=True)
    assert np.abs(in4.cpu().numpy() - o4).max() < ATOL
    check(logits.squeeze(-1).cpu().numpy(), dec.squeeze(-1).cpu().numpy(), d["logits"])
    assert out.shape == (y.shape[0], int(d["N"]), 2)
    # ragged batch over more than one 8192-codeword chunk
    rng = np.random.default_rng(2)
    yb = rng.standard_normal((8192 + 33, 64)).astype(np.float32)
    _, _, b4 = net.logits(torch.from_numpy(yb).to(DEV), want_input4=True)
    _, o4b = oracle.conv_forward(yb[::41], sd, want_input4=True)
    assert np.abs(b4.cpu().numpy()[::41] - o4b).max() < ATOL


# ------------------------------------------------------------------------------------------- fp16x3 conv layers
@pytest.mark.parametrize("name", ["conv_small_64", "conv_c5_256"])
def test_conv_fp16x3_golden(name):
    """precision "fp16x3" (conv layers with cin > 1 and the Linear layers on the fp16 MFMA, hi + lo split, 3 products
    per multiply, fp32 accumulation) held to the fp32 path's bars on the reference's golden logits: within 1e-5, decisions identical
    wherever the reference logit is farther than 1e-5 from zero (embed 16: 8-channel layers padded to 16; C5: embed
    128, N 256, 4 position tiles per wave)."""
    d = golden(f"{name}.npz")
    if "w.layer_norm.weight" in d.files:
        sd = {k[2:]: d[k] for k in d.files if k.startswith("w.")}
    else:
        sd = conv_weights_from_seed(int(d["embed"]), int(d["N"]), int(d["seed"]))
    net = net_from(sd, int(d["embed"]), int(d["N"]), precision="fp16x3")
    lg, dec = net.logits(torch.from_numpy(d["y"]).to(DEV))
    check(lg.cpu().numpy(), dec.cpu().numpy(), d["logits"])


def test_conv_fp16x3_error_matches_fp32_against_float64(oracle):
    """Precision study for the conv model (as tests/test_gru_precision_gpu.py for the GRU): |logit - float64 oracle|
    of the fp16x3 path against the fp32 path's on the same words, C5 shape (embed 128, N 256, seeded weights) and the
    trained embed-16 net: the fp16x3 error within 1.5 x the fp32 path's at p50 / p99 / p99.9 and its maximum within
    2 x (products to 2^-22 relative against fp32's exact products; both accumulate in fp32)."""
    rows = []
    d5 = golden("conv_c5_256.npz")
    sd5 = conv_weights_from_seed(int(d5["embed"]), int(d5["N"]), int(d5["seed"]))
    rng = np.random.default_rng(11)
    y5 = (np.where(rng.random((256, 256)) < 0.5, -1.0, 1.0) + 0.7 * rng.standard_normal((256, 256))).astype(np.float32)
    rows.append((sd5, int(d5["embed"]), 256, y5))
    import os
    tp = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "trained_conv_64_22.npz")
    if os.path.exists(tp):
        dt = np.load(tp)
        sdt = {k[2:]: np.asarray(dt[k]) for k in dt.files if k.startswith("w.")}
        yt = (np.where(rng.random((4096, 64)) < 0.5, -1.0, 1.0) + 0.8 * rng.standard_normal((4096, 64))).astype(np.float32)
        rows.append((sdt, int(dt["embed"]), 64, yt))
    for sd, E, N, y in rows:
        ref = oracle.conv_forward(y, sd).astype(np.float64)
        errs = {}
        for prec in ("fp32", "fp16x3"):
            lg, _ = net_from(sd, E, N, precision=prec).logits(torch.from_numpy(y).to(DEV))
            errs[prec] = np.abs(lg.cpu().numpy().astype(np.float64) - ref).ravel()
        q32 = np.percentile(errs["fp32"], [50, 99, 99.9])
        q16 = np.percentile(errs["fp16x3"], [50, 99, 99.9])
        print(E, N, "fp32", q32, errs["fp32"].max(), "fp16x3", q16, errs["fp16x3"].max())
        assert np.all(q16 <= 1.5 * q32), (E, N, q32, q16)
        assert errs["fp16x3"].max() <= 2.0 * errs["fp32"].max(), (E, N)


@pytest.mark.parametrize("E,N", [(64, 128), (64, 64), (80, 64), (96, 64), (128, 256)])
def test_conv_fp16x3_shapes_vs_oracle(oracle, E, N):
    """The fp16x3 kernels at every shape family they dispatch on, against the float64 oracle on a ragged batch of more
    than one 8192-codeword chunk (seeded weights, conftest.conv_weights_from_seed): embed 64 / N 128 (weight-stationary
    conv kernel with 32-channel groups, 128-position items; the 128 x 128 FC kernel for all three Linear layers); embed
    64 / N 64 (the 64-channel layer on 64-position items);
    embed 80 / N 64 (40-channel layers = three 16-channel groups, 64-position items; the 80-channel layer on the
    slab kernel; FC1 / FC2 of 64 outputs on the 64 x 64 FC kernel); embed 96 / N 64 (48-channel layers, the 96-channel
    layer on the slab kernel); C5 (embed 128, N 256: 64-channel layers on 4-wave blocks in 2 channel parts, the
    128-channel layer on 8 waves in 4). Same bars as the golden tests: logits within 1e-5, decisions identical away from
    zero."""
    sd = conv_weights_from_seed(E, N, 100 + E)
    net = net_from(sd, E, N, precision="fp16x3")
    rng = np.random.default_rng(E + N)
    B = 8192 + 37
    y = (np.where(rng.random((B, N)) < 0.5, -1.0, 1.0) + 0.8 * rng.standard_normal((B, N))).astype(np.float32)
    lg, dec = net.logits(torch.from_numpy(y).to(DEV))
    sel = np.r_[0:B:97, B - 1]
    ref = oracle.conv_forward(y[sel], sd)
    check(lg.cpu().numpy()[sel], dec.cpu().numpy()[sel], ref)


@pytest.mark.parametrize("E,N", [(64, 128), (128, 256), (80, 64)])
def test_conv_fp16x3_large_activations(oracle, E, N):
    """Activations far beyond fp16's range (received words x 3e4: conv and Linear inputs up to ~1e5): the split kernels
    scale each layer's input by 2^SA with SA from the producing kernel's max |a| (npd_conv.hip split_sa), so hi never
    overflows -- before that fix the fixed 2^4 scale turned every |a| > 4094 into inf and the logits into NaN.  The
    logits stay finite and match the float64 oracle (LayerNorm brings them back to O(1); 1e-4 absolute, the fp32 rounding of
    pre-LayerNorm values ~1e5 x 2^-24 relative to their spread) and the fp32 path's decisions."""
    sd = conv_weights_from_seed(E, N, 100 + E)
    rng = np.random.default_rng(5 + E)
    B = 257
    y = (3e4 * (np.where(rng.random((B, N)) < 0.5, -1.0, 1.0) + 0.8 * rng.standard_normal((B, N)))).astype(np.float32)
    lg16, dec16 = net_from(sd, E, N, precision="fp16x3").logits(torch.from_numpy(y).to(DEV))
    lg32, _ = net_from(sd, E, N, precision="fp32").logits(torch.from_numpy(y).to(DEV))
    lg16, lg32 = lg16.cpu().numpy(), lg32.cpu().numpy()
    assert np.isfinite(lg16).all()
    ref = oracle.conv_forward(y[::8], sd)
    assert np.abs(lg16[::8] - ref).max() < 1e-4, float(np.abs(lg16[::8] - ref).max())
    assert np.abs(lg16 - lg32).max() < 1e-4
    sure = np.abs(ref) > 1e-4
    assert np.array_equal(dec16.cpu().numpy()[::8][sure], np.sign(ref)[sure])


@pytest.mark.parametrize("var,v0,v1", [("NPD_FC0_PRESPLIT", "0", "1"), ("NPD_FC_BM", "128", "256")])
@pytest.mark.parametrize("E,N", [(128, 256), (64, 128)])
def test_conv_fc0_presplit_identical(monkeypatch, E, N, var, v0, v1):
    """NPD_FC0_PRESPLIT (default 0): FC0 reads X as fp16 hi / lo planes split once by split_planes_kernel (the same
    x 2^SA split the GEMM's loaders do otherwise) -- logits bit-identical to the in-loader split on a ragged batch of
    more than one chunk, and at activations beyond fp16's range (the planes carry the same 2^SA scaling).
    NPD_FC_BM (default: 256-row tiles where they fill every CU): the FC GEMM's 128- and 256-row block tiles sum every
    output over the same K order on the same 32 x 32 MFMA tiles, so the logits are bit-identical."""
    sd = conv_weights_from_seed(E, N, 100 + E)
    net = net_from(sd, E, N, precision="fp16x3")
    rng = np.random.default_rng(3 + E)
    for scale, B in ((1.0, 8192 + 19), (3e4, 129)):
        y = torch.from_numpy((scale * (np.where(rng.random((B, N)) < 0.5, -1.0, 1.0)
                                       + 0.8 * rng.standard_normal((B, N)))).astype(np.float32)).to(DEV)
        monkeypatch.setenv(var, v0)
        lg0, _ = net.logits(y)
        monkeypatch.setenv(var, v1)
        lg1, _ = net.logits(y)
        monkeypatch.delenv(var)
        assert torch.isfinite(lg1).all()
        assert torch.equal(lg0, lg1), float((lg0 - lg1).abs().max())


def test_conv_wide_shape_smaller_chunk_vs_oracle(oracle):
    """embed 128 / N 512 (FC0 K = 65536 into 2048 features): npd_conv_forward halves its 8192-codeword chunk while the
    three activation buffers would pass 4 GiB, so this batch runs in 4096-codeword chunks (the second one ragged);
    FC0's per-lane LDS / global offsets stay block-relative at this K.  fp16x3 and fp32 against the float64
    oracle on rows of both chunks, the same bars as the other shapes."""
    E, N = 128, 512
    sd = conv_weights_from_seed(E, N, 7)
    rng = np.random.default_rng(17)
    B = 4096 + 21
    y = (np.where(rng.random((B, N)) < 0.5, -1.0, 1.0) + 0.8 * rng.standard_normal((B, N))).astype(np.float32)
    sel = np.array([0, 2047, 4095, 4096, B - 1])
    ref = oracle.conv_forward(y[sel], sd)
    for prec in ("fp16x3", "fp32"):
        lg, dec = net_from(sd, E, N, precision=prec).logits(torch.from_numpy(y).to(DEV))
        check(lg.cpu().numpy()[sel], dec.cpu().numpy()[sel], ref)
