"""--use_layernorm nets (rnn_all.py:317-320; forward rnn_all.py:387-398: decoded = linear(layernorm(out))) on the CPU:
the float64 oracle (oracle.gru_decode_f64 with ln_eps; y_h0 through oracle.ymlp_f64) against the reference's golden
decisions and logits (tests/golden/gen_golden.py gen_gru_ln: y_input at hidden 64 x 2 layers and hidden 32 x 1 layer with
sign input and reverse order, y_h0 at hidden 32 x 2 layers; LayerNorm gamma / beta drawn away from (1, 0)), and the
fused decoder's support rule (fp32 GRU, hidden 32 / 64, unidirectional)."""
import numpy as np
import pytest
import torch

from conftest import golden

CASES = ["gru_ln_polar_32_16", "gru_ln_polar_16_8_l1_noonehot_rev", "gru_ln_yh0_polar_32_16_f32"]


def load(name):
    d = golden(f"{name}.npz")
    return d, {k[2:]: d[k] for k in d.files if k.startswith("w.")}


def model(d):
    from neural_polar_decoder_amd.rnn import RNN_Model
    N, F, L = int(d["N"]), int(d["F"]), int(d["layers"])
    yin = bytes(d["decoding_type"]).decode() == "y_input"
    return RNN_Model("GRU", (N if yin else 0) + 1 + int(d["onehot"]), F, 1, L, N, int(d["y_hidden"]), int(d["y_depth"]),
                     bytes(d["activation"]).decode(), 0.0, False, use_layernorm=True)


@pytest.mark.parametrize("name", CASES)
def test_oracle_ln_matches_reference(oracle, name):
    d, sd = load(name)
    N, F, L = int(d["N"]), int(d["F"]), int(d["layers"])
    h0x = None
    if bytes(d["decoding_type"]).decode() == "y_h0":
        h0x = oracle.ymlp_f64(d["y"], sd, bytes(d["activation"]).decode(), int(d["y_depth"]))
    dec, lg = oracle.gru_decode_f64(d["y"], sd, N, F, L, d["info"], onehot=bool(d["onehot"]), h0x=h0x,
                                    rev=bool(d["rev"]), ln_eps=float(d["ln_eps"]))
    info = d["info"]
    ref = d["decoded"]
    assert (dec[:, info] == ref[:, info]).mean() >= 0.999
    same = (dec[:, info] == ref[:, info]).all(1)
    assert same.mean() >= 0.99
    assert np.abs(lg[same] - d["logits"][same]).max() < 2e-5
    # the LayerNorm matters: without it the same weights give other logits
    _, lg0 = oracle.gru_decode_f64(d["y"][:64], sd, N, F, L, info, onehot=bool(d["onehot"]),
                                   h0x=None if h0x is None else h0x[:64], rev=bool(d["rev"]))
    assert np.abs(lg0 - d["logits"][:64]).max() > 1e-2


@pytest.mark.parametrize("name", CASES)
def test_ln_model_loads_and_support_rule(name):
    d, sd = load(name)
    net = model(d)
    net.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
    dt = bytes(d["decoding_type"]).decode()
    assert net.fused_supported(dt, "fp32", int(d["N"]))
    assert not net.fused_supported(dt, "fp16x3", int(d["N"]))  # the LayerNorm head runs on the fp32 kernel only


def test_ln_support_excludes_other_kernels():
    from neural_polar_decoder_amd.rnn import RNN_Model
    assert not RNN_Model("GRU", 66, 128, 1, 2, 64, 0, 0, use_layernorm=True).fused_supported("y_input")  # hidden 128
    assert not RNN_Model("LSTM", 66, 64, 1, 1, 64, 0, 0, use_layernorm=True).fused_supported("y_input")
    assert not RNN_Model("GRU", 66, 32, 1, 2, 64, 0, 0, bidirectional=True,
                         use_layernorm=True).fused_supported("y_input")
    # a LayerNorm in front of an out_linear_depth > 1 head is not fused
    assert not RNN_Model("GRU", 66, 64, 1, 2, 64, 64, 0, out_linear_depth=2,
                         use_layernorm=True).fused_supported("y_input")
