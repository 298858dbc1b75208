"""decoding_type 'y_h0' on the MI355X (rnn_all.py:523-531): the y-MLP on npd_ymlp_layer and the GRU decode from its
initial states (npd_gru_decode_ex, y = NULL) against the reference's golden decisions / logits / initial states
(tests/golden/gen_golden.py gen_gru_yh0), the same bars as the y_input fixtures: >= 99.9 % of information bits and
>= 99 % of codewords identical, logits of agreeing codewords within 2e-5; fp32 kernels (F 32 / 64, and F 128 on the
weight-streaming kernel) and the fp16x3 split (F = 64, 2 layers, N % 32 == 0)."""
import numpy as np
import pytest
import torch

from conftest import golden

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
CASES = ["gru_yh0_polar_64_32", "gru_yh0_polar_32_16_f128_relu_rev", "gru_yh0_polar_16_8_l1_tanh_noonehot",
         "gru_yh0_polar_32_16_elu_d1", "gru_yh0_polar_16_8_sigmoid", "gru_yh0_polar_32_16_skip"]
SPLIT_OK = {"gru_yh0_polar_64_32", "gru_yh0_polar_32_16_elu_d1", "gru_yh0_polar_32_16_skip"}


def build(name, precision="fp32"):
    from neural_polar_decoder_amd.rnn import RNN_decoder, RNN_Model
    d = golden(f"{name}.npz")
    sd = {k[2:]: torch.from_numpy(d[k]) for k in d.files if k.startswith("w.")}
    N, F, L = int(d["N"]), int(d["F"]), int(d["layers"])
    skip = bool(int(d["skip"])) if "skip" in d.files else False  # gen_gru_yh0_skip (rnn_all.py:369-370)
    net = RNN_Model("GRU", 1 + int(d["onehot"]), F, 1, L, N, int(d["y_hidden"]), int(d["y_depth"]),
                    bytes(d["activation"]).decode(), 0.0, skip).to(DEV).eval()
    net.load_state_dict(sd)
    dec = RNN_decoder("y_h0", N, d["info"], onehot=bool(d["onehot"]), reverse_order=bool(d["rev"]),
                      precision=precision)
    return d, net, dec


@pytest.mark.parametrize("precision", ["fp32", "fp16x3"])
@pytest.mark.parametrize("name", CASES)
def test_yh0_decode_matches_reference(name, precision):
    if precision != "fp32" and name not in SPLIT_OK:
        pytest.skip("the split paths with an initial state run on the 16-codeword kernel (F = 64, 2 layers)")
    d, net, dec = build(name, precision)
    info = d["info"]
    out, lg = dec.decode(net, False, torch.from_numpy(d["y"]).to(DEV), return_logits=True)
    got = out.cpu().numpy()
    assert (got[:, info] == d["decoded"][:, info]).mean() >= 0.999
    same = (got[:, info] == d["decoded"][:, info]).all(1)
    assert same.mean() >= 0.99
    assert np.abs(lg.cpu().numpy()[same] - d["logits"][same]).max() < 2e-5
    frozen = np.setdiff1d(np.arange(int(d["N"])), info)
    assert np.all(got[:, frozen] == 1.0)


@pytest.mark.parametrize("name", CASES)
def test_yh0_mlp_matches_reference(name):
    d, net, dec = build(name)
    x = dec._h0(net, torch.from_numpy(d["y"]).to(DEV)).cpu().numpy()  # the MLP (and skip's y in front) on the GPU
    assert np.abs(x - d["h0x"]).max() < 1e-5


def test_yh0_ragged_batch_vs_oracle(oracle):
    """More words than one grid pass, ragged, against the float64 oracle on a sample of rows."""
    d, net, dec = build("gru_yh0_polar_64_32")
    sd = {k[2:]: d[k] for k in d.files if k.startswith("w.")}
    rng = np.random.default_rng(7)
    B = 70001
    y = (np.where(rng.random((B, 64)) < 0.5, -1.0, 1.0) + 0.9 * rng.standard_normal((B, 64))).astype(np.float32)
    out, lg = dec.decode(net, False, torch.from_numpy(y).to(DEV), return_logits=True)
    sel = np.r_[0:B:499, B - 1]
    x = oracle.ymlp_f64(y[sel], sd, "selu", int(d["y_depth"]))
    dref, lref = oracle.gru_decode_f64(y[sel], sd, 64, 64, 2, d["info"], onehot=True, h0x=x)
    info = d["info"]
    got = out.cpu().numpy()[sel]
    same = (got[:, info] == dref[:, info]).all(1)
    assert same.mean() >= 0.99
    assert np.abs(lg.cpu().numpy()[sel][same] - lref[same]).max() < 2e-5


def test_yh0_unsupported_split_shape_raises():
    from neural_polar_decoder_amd import _lib
    d, net, dec = build("gru_yh0_polar_16_8_sigmoid", precision="bf16x3")
    with pytest.raises(_lib.NpdError):
        dec.decode(net, False, torch.from_numpy(d["y"]).to(DEV))
