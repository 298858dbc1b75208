"""--use_ynn decoding on the MI355X (rnn_all.py:533-536): the y-MLP on npd_ymlp_layer, its N outputs fed to the fused
y_input kernels in place of y, against the reference's golden decisions / logits / Fy (tests/golden/gen_golden.py
gen_gru_ynn), the y_input fixtures' bars: >= 99.9 % of information bits and >= 99 % of codewords identical, logits
of agreeing codewords within 2e-5; fp32 kernels and the fp16x3 split (F = 64, 2 layers, N % 32 == 0)."""
import numpy as np
import pytest
import torch

from conftest import golden

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
CASES = ["gru_ynn_polar_64_32", "gru_ynn_polar_32_16_f32_tanh_rev", "gru_ynn_polar_16_8_d1_noonehot"]
SPLIT_OK = {"gru_ynn_polar_64_32"}


def build(name, precision="fp32"):
    from neural_polar_decoder_amd.rnn import RNN_decoder, RNN_Model
    d = golden(f"{name}.npz")
    N, F, L = int(d["N"]), int(d["F"]), int(d["layers"])
    net = RNN_Model("GRU", N + 1 + int(d["onehot"]), F, 1, L, N, int(d["y_hidden"]), int(d["y_depth"]),
                    bytes(d["activation"]).decode(), 0.0, False, y_output_size=N).to(DEV).eval()
    net.load_state_dict({k[2:]: torch.from_numpy(d[k]) for k in d.files if k.startswith("w.")})
    dec = RNN_decoder("y_input", N, d["info"], onehot=bool(d["onehot"]), reverse_order=bool(d["rev"]),
                      precision=precision)
    return d, net, dec


@pytest.mark.parametrize("precision", ["fp32", "fp16x3"])
@pytest.mark.parametrize("name", CASES)
def test_ynn_decode_matches_reference(name, precision):
    if precision != "fp32" and name not in SPLIT_OK:
        pytest.skip("the unscaled split runs on the 16-codeword kernel (F = 64, 2 layers, N % 32 == 0)")
    d, net, dec = build(name, precision)
    info = d["info"]
    out, lg = dec.decode(net, False, torch.from_numpy(d["y"]).to(DEV), return_logits=True)
    got = out.cpu().numpy()
    assert (got[:, info] == d["decoded"][:, info]).mean() >= 0.999
    same = (got[:, info] == d["decoded"][:, info]).all(1)
    assert same.mean() >= 0.99
    assert np.abs(lg.cpu().numpy()[same] - d["logits"][same]).max() < 2e-5


@pytest.mark.parametrize("name", CASES)
def test_ynn_mlp_matches_reference(name):
    from neural_polar_decoder_amd.rnn import _ymlp_forward
    d, net, _ = build(name)
    fy = _ymlp_forward(net, torch.from_numpy(d["y"]).to(DEV)).cpu().numpy()
    assert np.abs(fy - d["fy"]).max() < 1e-5


def test_ynn_ragged_batch_vs_oracle(oracle):
    """More words than one grid pass, ragged, against the float64 oracle (ymlp_f64 + gru_decode_f64) on sampled rows."""
    d, net, dec = build("gru_ynn_polar_64_32")
    sd = {k[2:]: d[k] for k in d.files if k.startswith("w.")}
    rng = np.random.default_rng(3)
    B = 70000 + 13
    y = (np.where(rng.random((B, 64)) < 0.5, -1.0, 1.0) + 0.9 * rng.standard_normal((B, 64))).astype(np.float32)
    out, lg = dec.decode(net, False, torch.from_numpy(y).to(DEV), return_logits=True)
    sel = np.r_[0:B:211, B - 1]
    fy = oracle.ymlp_f64(y[sel], sd, bytes(d["activation"]).decode(), int(d["y_depth"]))
    ref, rlg = oracle.gru_decode_f64(fy, sd, 64, int(d["F"]), int(d["layers"]), d["info"], onehot=True)
    info = d["info"]
    got = out.cpu().numpy()[sel]
    same = (got[:, info] == ref[:, info]).all(1)
    assert same.mean() >= 0.99
    assert np.abs(lg.cpu().numpy()[sel][same] - rlg[same]).max() < 2e-5
