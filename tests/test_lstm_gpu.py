"""LSTM cells on the MI355X (lstm_decode_kernel, fp32): RNN_decoder.decode(net, False, y) for an nn.LSTM net against
the reference's golden decisions and logits (tests/golden/gen_golden.py gen_lstm), the y_input fixtures' bars:
>= 99.9 % of information bits and >= 99 % of codewords identical, logits of agreeing codewords within 2e-5; a
ragged multi-pass batch against the float64 oracle."""
import numpy as np
import pytest
import torch

from conftest import golden

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
CASES = ["lstm_polar_64_32_f64_l1", "lstm_polar_32_16_f32_l2_rev", "lstm_polar_16_8_f32_l1_noonehot"]


def build(name):
    from neural_polar_decoder_amd.rnn import RNN_decoder, RNN_Model
    d = golden(f"{name}.npz")
    N, F, L = int(d["N"]), int(d["F"]), int(d["layers"])
    net = RNN_Model("LSTM", N + 1 + int(d["onehot"]), F, 1, L, N, 0, 0).to(DEV).eval()
    net.load_state_dict({k[2:]: torch.from_numpy(d[k]) for k in d.files if k.startswith("w.")})
    return d, net, RNN_decoder("y_input", N, d["info"], onehot=bool(d["onehot"]), reverse_order=bool(d["rev"]))


@pytest.mark.parametrize("name", CASES)
def test_lstm_decode_matches_reference(name):
    d, net, dec = build(name)
    info = d["info"]
    out, lg = dec.decode(net, False, torch.from_numpy(d["y"]).to(DEV), return_logits=True)
    got = out.cpu().numpy()
    assert (got[:, info] == d["decoded"][:, info]).mean() >= 0.999
    same = (got[:, info] == d["decoded"][:, info]).all(1)
    assert same.mean() >= 0.99
    assert np.abs(lg.cpu().numpy()[same] - d["logits"][same]).max() < 2e-5


def test_lstm_ragged_batch_vs_oracle(oracle):
    d, net, dec = build("lstm_polar_32_16_f32_l2_rev")
    sd = {k[2:]: d[k] for k in d.files if k.startswith("w.")}
    rng = np.random.default_rng(9)
    B = 50001
    y = (np.where(rng.random((B, 32)) < 0.5, -1.0, 1.0) + 0.9 * rng.standard_normal((B, 32))).astype(np.float32)
    out, lg = dec.decode(net, False, torch.from_numpy(y).to(DEV), return_logits=True)
    sel = np.r_[0:B:401, B - 1]
    dref, lref = oracle.gru_decode_f64(y[sel], sd, 32, 32, 2, d["info"], onehot=True, rev=True, cell="LSTM")
    info = d["info"]
    same = (out.cpu().numpy()[sel][:, info] == dref[:, info]).all(1)
    assert same.mean() >= 0.99
    assert np.abs(lg.cpu().numpy()[sel][same] - lref[same]).max() < 2e-5
