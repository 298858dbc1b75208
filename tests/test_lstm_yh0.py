"""LSTM cells with decoding_type y_h0 (rnn_all.py:69 --rnn_type LSTM, decode test branch rnn_all.py:523-531; get_h0
returns (x, x) for LSTM, so h and c both start from the y-MLP's output, rnn_all.py:370-375): the float64 oracle
(oracle.ymlp_f64 + gru_decode_f64(cell="LSTM", h0x=...)) against the reference's golden decisions, logits and initial
states (tests/golden/gen_golden.py gen_lstm_yh0: seeded PyTorch-default weights; hidden 32 with 2 layers, hidden 64
with 1 layer in reverse order), and the same decode on the MI355X (lstm_decode_kernel from initial states) under the
y_input fixtures' bars."""
import numpy as np
import pytest
import torch

from conftest import golden

CASES = ["lstm_yh0_polar_32_16_f32_l2", "lstm_yh0_polar_64_32_f64_l1_tanh_rev"]


def load(name):
    d = golden(f"{name}.npz")
    sd = {k[2:]: d[k] for k in d.files if k.startswith("w.")}
    return d, sd


@pytest.mark.parametrize("name", CASES)
def test_oracle_lstm_yh0_matches_reference(oracle, name):
    d, sd = load(name)
    N, F, L = int(d["N"]), int(d["F"]), int(d["layers"])
    x = oracle.ymlp_f64(d["y"], sd, bytes(d["activation"]).decode(), int(d["y_depth"]))
    assert np.abs(x - d["h0x"]).max() < 1e-5
    dec, lg = oracle.gru_decode_f64(d["y"], sd, N, F, L, d["info"], onehot=bool(d["onehot"]), h0x=x,
                                    rev=bool(d["rev"]), cell="LSTM")
    info = d["info"]
    assert (dec[:, info] == d["decoded"][:, info]).mean() >= 0.999
    same = (dec[:, info] == d["decoded"][:, info]).all(1)
    assert same.mean() >= 0.99
    assert np.abs(lg[same] - d["logits"][same]).max() < 2e-5


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_lstm_yh0_decode_matches_reference(name):
    from neural_polar_decoder_amd.rnn import RNN_decoder, RNN_Model
    d, sd = load(name)
    N, F, L = int(d["N"]), int(d["F"]), int(d["layers"])
    net = RNN_Model("LSTM", 1 + int(d["onehot"]), F, 1, L, N, int(d["y_hidden"]), int(d["y_depth"]),
                    bytes(d["activation"]).decode(), 0.0, False).to("cuda:0").eval()
    net.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    assert net.fused_supported("y_h0")
    dec = RNN_decoder("y_h0", N, d["info"], onehot=bool(d["onehot"]), reverse_order=bool(d["rev"]))
    out, lg = dec.decode(net, False, torch.from_numpy(d["y"]).to("cuda:0"), return_logits=True)
    info = d["info"]
    got = out.cpu().numpy()
    assert (got[:, info] == d["decoded"][:, info]).mean() >= 0.999
    same = (got[:, info] == d["decoded"][:, info]).all(1)
    assert same.mean() >= 0.99
    assert np.abs(lg.cpu().numpy()[same] - d["logits"][same]).max() < 2e-5
