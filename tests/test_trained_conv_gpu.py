"""The fused convNet decoder (npd_conv_forward) at trained-model margins.

Fixtures: tests/golden/trained_conv_64_22.npz -- a convNet (embed 16, Polar(64,22) 'polar' profile) trained with the
reference's own run_models.py over run_alt.sh's n2c curriculum shape (tests/golden/gen_trained_conv.py) -- and
trained_conv_64_22_e128.npz, run_alt.sh's own width (embed 128, batch 8192; stages on the GPU by
tests/golden/train_conv_gpu.py): the reference's decisions and logits on the fixture words per SNR (0..4 dB) and its
Monte-Carlo BER/BLER curve (2^18 words per SNR through convNet.decode on the CPU).

Tolerance (as tests/test_conv_gpu.py for logits, as tests/test_trained_gru_gpu.py for the curve):
  (a) decisions on the fixture words: >= 99.9 % of information bits and >= 99 % of codewords identical to the
      reference's; logits within 1e-4 absolute (ATOL: the trained net's reference fp32 logits themselves sit up to
      3.1e-5 from float64, so the seeded nets' 1e-5 bar of tests/test_conv_gpu.py does not apply);
  (b) Monte-Carlo at 2^18 Philox words per SNR: BLER and BER within 4 two-sample standard errors of the reference's
      curve, and the BLER curve's horizontal offset within +-0.05 dB at every point whose reference BLER is in
      [1e-3, 0.9] and where the two samples resolve it (3 sigma_dB <= 0.05; elsewhere in that domain within 3 sigma),
      at >= 2 such points (conftest.assert_db_bar, as tests/test_trained_gru_gpu.py).
"""
import argparse

import numpy as np
import pytest
import torch

from conftest import assert_db_bar, trained_fixture

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
ATOL = 1e-4  # trained weights: the reference's fp32 logits are up to 3.1e-5 from float64 (tests/test_trained_conv.py)
# embed 16 (the reference's run_models.py for every stage) and run_alt.sh's own embed 128 (round 6: every stage on the
# GPU, tests/golden/train_conv_gpu.py; the configs[4] kernel family -- 64-channel conv_ws16 layers, the 128-channel
# layer, the 128-tile FC GEMM)
NAMES = ["trained_conv_64_22", "trained_conv_64_22_e128"]


def net_from(d, precision="fp32"):
    from neural_polar_decoder_amd.models import convNet
    N = int(d["N"])
    cfg = argparse.Namespace(embed_dim=int(d["embed"]), max_len=N, N=N, dont_use_bias=False, dropout=0.0)
    net = convNet(cfg, precision=precision)
    net.load_state_dict({k[2:]: torch.from_numpy(np.asarray(d[k])) for k in d.files if k.startswith("w.")})
    return net.eval()


def fixture_words(d, si):
    """The fixture's words at SNR index si, regenerated as gen_trained_conv.py drew them through the reference
    (torch.manual_seed(seed_dec + si); msg = 1 - 2 (rand < 0.5); y = encode_plotkin(msg) + sigma randn) with the
    oracle's bit-exact encoder, checked against the stored sha256."""
    import hashlib
    from oracle import oracle as O
    N, K = int(d["N"]), int(d["K"])
    torch.manual_seed(int(d["seed_dec"]) + si)
    msg = 1.0 - 2.0 * (torch.rand(int(d["n_dec"]), K) < 0.5).float()
    x = torch.from_numpy(O.encode_plotkin(msg.numpy(), N, d["info"]))
    y = (x + 10 ** (-float(d["snr"][si]) / 20) * torch.randn(x.shape, dtype=torch.float)).numpy()
    assert hashlib.sha256(np.ascontiguousarray(y).tobytes()).hexdigest() == bytes(d[f"y_digest_{si}"]).decode()
    return msg.numpy(), y


@pytest.mark.parametrize("precision", ["fp32", "fp16x3"])
@pytest.mark.parametrize("name", NAMES)
def test_trained_conv_decisions_match_reference(name, precision):
    d = trained_fixture(name)
    net = net_from(d, precision)
    N, K = int(d["N"]), int(d["K"])
    info = d["info"]
    for si in range(len(d["snr"])):
        _, y = fixture_words(d, si)
        lg, dec = net.logits(torch.from_numpy(y).to(DEV))
        got = dec.view(-1, N).cpu().numpy()[:, info]
        ref = np.where(np.unpackbits(d[f"dec_bits_{si}"], axis=1)[:, :K] == 1, -1.0, 1.0)
        assert (got == ref).mean() >= 0.999
        assert (got == ref).all(1).mean() >= 0.99
        m = d[f"logits_{si}"].shape[0]
        assert np.abs(lg.view(-1, N).cpu().numpy()[:m] - d[f"logits_{si}"]).max() < ATOL


@pytest.mark.parametrize("precision", ["fp32", "fp16x3"])
@pytest.mark.parametrize("name", NAMES)
def test_trained_conv_ber_curve_matches_reference(name, precision):
    from neural_polar_decoder_amd import reference_polar_code
    d = trained_fixture(name)
    net = net_from(d, precision)
    N, K = int(d["N"]), int(d["K"])
    code = reference_polar_code(N, K)
    assert np.array_equal(np.asarray(code.info_positions), d["info"])
    info = torch.as_tensor(d["info"], device=DEV)
    snrs = [float(s) for s in d["snr"]]
    n, nr = 1 << 18, int(d["mc_n"])
    bler = []
    for si, s in enumerate(snrs):
        be = bl = sq = 0
        for off in range(0, n, 1 << 16):
            msg, _, y = code.mc_generate(1 << 16, s, 2029, si, off, device=DEV)
            _, dec = net.logits(y)
            e = (dec.view(-1, N)[:, info] != msg).sum(1).to(torch.int64)
            be, bl, sq = be + int(e.sum()), bl + int((e > 0).sum()), sq + int((e * e).sum())
        rbe, rbl, rsq = int(d["mc_bit_err"][si]), int(d["mc_blk_err"][si]), int(d["mc_sq_err"][si])
        p, pr = bl / n, rbl / nr
        pool = (bl + rbl) / (n + nr)
        z_bler = (p - pr) / np.sqrt(max(pool * (1 - pool), 1e-300) * (1 / n + 1 / nr))
        v, vr = sq / n - (be / n) ** 2, rsq / nr - (rbe / nr) ** 2
        z_ber = (be / n - rbe / nr) / np.sqrt(max(v / n + vr / nr, 1e-300))
        assert abs(z_bler) < 4 and abs(z_ber) < 4, (s, p, pr, z_bler, z_ber)
        bler.append(p)
    ref_bler = [int(x) / nr for x in d["mc_blk_err"]]
    # +-0.05 dB where resolvable (at ref BLER ~1e-3 the two 2^18-word samples leave sigma_dB ~0.04: within 3 sigma)
    assert_db_bar(snrs, bler, n, ref_bler, nr)
