"""--rnn_type LSTM (rnn_all.py:69), decoding_type y_input (rnn_all.py:532-547) on the CPU: the float64 oracle's LSTM
step against the reference's golden decisions and logits (tests/golden/gen_golden.py gen_lstm: seeded PyTorch-default
weights; hidden 64 / 1 layer, hidden 32 / 2 layers reversed, hidden 32 / sign input)."""
import numpy as np
import pytest

from conftest import golden

CASES = ["lstm_polar_64_32_f64_l1", "lstm_polar_32_16_f32_l2_rev", "lstm_polar_16_8_f32_l1_noonehot"]


@pytest.mark.parametrize("name", CASES)
def test_oracle_lstm_matches_reference(oracle, name):
    d = golden(f"{name}.npz")
    sd = {k[2:]: d[k] for k in d.files if k.startswith("w.")}
    N, F, L = int(d["N"]), int(d["F"]), int(d["layers"])
    dec, lg = oracle.gru_decode_f64(d["y"], sd, N, F, L, d["info"], onehot=bool(d["onehot"]), rev=bool(d["rev"]),
                                    cell="LSTM")
    info = d["info"]
    ref = d["decoded"]
    assert (dec[:, info] == ref[:, info]).mean() >= 0.999
    same = (dec[:, info] == ref[:, info]).all(1)
    assert same.mean() >= 0.99
    assert np.abs(lg[same] - d["logits"][same]).max() < 2e-5


def test_lstm_shapes_accepted():
    import torch
    from neural_polar_decoder_amd.rnn import RNN_Model
    assert RNN_Model("LSTM", 66, 64, 1, 1, 64, 0, 0).fused_supported("y_input")
    assert RNN_Model("LSTM", 34, 32, 1, 2, 32, 0, 0).fused_supported("y_input")
    assert RNN_Model("LSTM", 66, 64, 1, 2, 64, 0, 0).fused_supported("y_input")  # lstm_wide_kernel (round 5)
    assert RNN_Model("LSTM", 66, 256, 1, 2, 64, 0, 0).fused_supported("y_input")
    assert not RNN_Model("LSTM", 66, 96, 1, 1, 64, 0, 0).fused_supported("y_input")
    assert RNN_Model("LSTM", 2, 32, 1, 1, 32, 64, 2).fused_supported("y_h0")  # y_h0: (h, c) = (x, x), round 5
    assert RNN_Model("LSTM", 2, 64, 1, 2, 64, 64, 2).fused_supported("y_h0")
    del torch
