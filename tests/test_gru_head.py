"""--out_linear_depth > 1 heads (rnn_all.py:336-343: Linear(F, H), SELU, [Linear(H, H), SELU] ..., Linear(H, 1); y_input
nets as rnn_all.py:1320 builds them) on the CPU: the float64 oracle (oracle.gru_decode_f64 runs the Sequential head)
against the reference's golden decisions and logits (tests/golden/gen_golden.py gen_gru_head: depth 2 / 3, H 48 / 64 /
128, hidden 32 / 64, 1 / 2 layers, one-hot and sign input, reverse order), the package's RNN_Model loading the
reference's head parameters, and the fused decoder's support rule."""
import numpy as np
import pytest
import torch

from conftest import golden

CASES = ["gru_head_polar_32_16_d2_h64", "gru_head_polar_16_8_d3_h48_noonehot_rev", "gru_head_polar_32_16_f32_d2_h128",
         "gru_head_bi_polar_32_16_f32_d2_h64"]


def load(name):
    d = golden(f"{name}.npz")
    return d, {k[2:]: d[k] for k in d.files if k.startswith("w.")}


def bi(d):
    return "bidirectional" in d.files and int(d["bidirectional"]) == 1


def model(d):
    from neural_polar_decoder_amd.rnn import RNN_Model
    N, F, L = int(d["N"]), int(d["F"]), int(d["layers"])
    return RNN_Model("GRU", N + 1 + int(d["onehot"]), F, 1, L, N, int(d["y_hidden"]), 0, "selu", 0.0, False,
                     out_linear_depth=int(d["out_linear_depth"]), bidirectional=bi(d))


@pytest.mark.parametrize("name", CASES)
def test_oracle_head_matches_reference(oracle, name):
    d, sd = load(name)
    N, F, L = int(d["N"]), int(d["F"]), int(d["layers"])
    if bi(d):  # the packed 2F cell (tests/test_rnn_bi.py) under the Sequential head, which reads [h_fwd, h_rev]
        from test_rnn_bi import packed_state_dict
        net = model(d)
        net.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
        psd = packed_state_dict(net)
        psd = {k: v for k, v in psd.items() if not k.startswith("linear.")}
        psd.update({k: v for k, v in sd.items() if k.startswith("linear.")})
        sd, F = psd, 2 * F
    dec, lg = oracle.gru_decode_f64(d["y"], sd, N, F, L, d["info"], onehot=bool(d["onehot"]), rev=bool(d["rev"]))
    info = d["info"]
    ref = d["decoded"]
    assert (dec[:, info] == ref[:, info]).mean() >= 0.999
    same = (dec[:, info] == ref[:, info]).all(1)
    assert same.mean() >= 0.99
    assert np.abs(lg[same] - d["logits"][same]).max() < 2e-5


@pytest.mark.parametrize("name", CASES)
def test_head_model_loads_and_support_rule(name):
    from neural_polar_decoder_amd.rnn import pack_head_weights
    d, sd = load(name)
    N, F, depth, H = int(d["N"]), int(d["F"]), int(d["out_linear_depth"]), int(d["y_hidden"])
    net = model(d)
    net.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
    assert net.fused_supported("y_input", "fp32", N)
    assert not net.fused_supported("y_input", "fp16x3", N)
    hw = pack_head_weights(net)
    Fi = F * (2 if bi(d) else 1)
    assert hw.size == H * Fi + H + (depth - 2) * (H * H + H) + H + 1


def test_head_support_limits():
    from neural_polar_decoder_amd.rnn import RNN_Model
    assert not RNN_Model("GRU", 66, 128, 1, 2, 64, 64, 0, out_linear_depth=2).fused_supported("y_input")  # hidden 128
    assert not RNN_Model("GRU", 66, 64, 1, 2, 64, 256, 0, out_linear_depth=2).fused_supported("y_input")  # H > 128
    assert not RNN_Model("LSTM", 66, 64, 1, 1, 64, 64, 0, out_linear_depth=2).fused_supported("y_input")
    assert not RNN_Model("GRU", 66, 64, 1, 2, 64, 64, 0, out_linear_depth=2,
                         use_layernorm=True).fused_supported("y_input")
