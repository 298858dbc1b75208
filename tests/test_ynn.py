"""decoding_type 'y_input' with --use_ynn (rnn_all.py:1319-1320; decode test branch rnn_all.py:533-536: Fy = get_Fy(y),
the y-MLP's N outputs replacing y as the GRU input) on the CPU: the float64 oracle (oracle.ymlp_f64 + gru_decode_f64 on
Fy) and this package's RNN_Model.get_Fy against the reference's golden decisions, logits and Fy
(tests/golden/gen_golden.py gen_gru_ynn: PyTorch-default seeded weights; selu / tanh / relu, 1 / 2 layers, F 32 / 64,
one-hot and sign inputs, reverse order, y_depth 1..3), and the reference checkpoint format through
datasets.rnn_from_checkpoint."""
import argparse

import numpy as np
import pytest
import torch

from conftest import golden

CASES = ["gru_ynn_polar_64_32", "gru_ynn_polar_32_16_f32_tanh_rev", "gru_ynn_polar_16_8_d1_noonehot"]


def load(name):
    d = golden(f"{name}.npz")
    sd = {k[2:]: d[k] for k in d.files if k.startswith("w.")}
    return d, sd


def model(d, sd):
    from neural_polar_decoder_amd.rnn import RNN_Model
    N, F, L = int(d["N"]), int(d["F"]), int(d["layers"])
    net = RNN_Model("GRU", N + 1 + int(d["onehot"]), F, 1, L, N, int(d["y_hidden"]), int(d["y_depth"]),
                    bytes(d["activation"]).decode(), 0.0, False, y_output_size=N)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    return net.eval()


@pytest.mark.parametrize("name", CASES)
def test_oracle_ynn_matches_reference(oracle, name):
    d, sd = load(name)
    N, F, L = int(d["N"]), int(d["F"]), int(d["layers"])
    fy = oracle.ymlp_f64(d["y"], sd, bytes(d["activation"]).decode(), int(d["y_depth"]))
    assert np.abs(fy - d["fy"]).max() < 1e-5  # the reference's fp32 MLP against float64
    dec, lg = oracle.gru_decode_f64(fy, sd, N, F, L, d["info"], onehot=bool(d["onehot"]), rev=bool(d["rev"]))
    info = d["info"]
    ref = d["decoded"]
    assert (dec[:, info] == ref[:, info]).mean() >= 0.999
    same = (dec[:, info] == ref[:, info]).all(1)
    assert same.mean() >= 0.99
    assert np.abs(lg[same] - d["logits"][same]).max() < 2e-5


@pytest.mark.parametrize("name", CASES)
def test_rnn_model_get_fy_matches_reference(name):
    d, sd = load(name)
    net = model(d, sd)
    assert net.fused_supported("y_input")
    with torch.no_grad():
        fy = net.get_Fy(torch.from_numpy(d["y"])).numpy()
    assert np.abs(fy - d["fy"]).max() < 1e-6


def test_rnn_from_checkpoint_use_ynn():
    """A --use_ynn checkpoint ({'net', 'args'}) builds the reference's module set (rnn_all.py:1319: y_output_size = N)."""
    from neural_polar_decoder_amd.datasets import rnn_from_checkpoint
    d, sd = load("gru_ynn_polar_64_32")
    args = argparse.Namespace(decoding_type="y_input", use_ynn=True, onehot=True, N=64, K=32, rnn_feature_size=64,
                              rnn_depth=2, y_hidden_size=int(d["y_hidden"]), y_depth=int(d["y_depth"]),
                              activation=bytes(d["activation"]).decode(), code="Polar", rate_profile="polar",
                              target_K=32, rnn_type="GRU", out_linear_depth=1)
    net, dec, code = rnn_from_checkpoint({"net": {k: torch.from_numpy(v) for k, v in sd.items()}, "args": args},
                                         device="cpu")
    assert dec.decoding_type == "y_input" and net.fused_supported("y_input") and net.y_output_size == 64
    with torch.no_grad():
        fy = net.get_Fy(torch.from_numpy(d["y"])).numpy()
    assert np.abs(fy - d["fy"]).max() < 1e-6
