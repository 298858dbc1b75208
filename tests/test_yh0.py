"""decoding_type 'y_h0' (rnn_all.py:73 default; decode test branch rnn_all.py:523-531) on the CPU: the float64 oracle
(oracle.ymlp_f64 + gru_decode_f64 with an initial state) and this package's RNN_Model.get_h0 against the reference's
golden decisions, logits and initial states (tests/golden/gen_golden.py gen_gru_yh0: PyTorch-default seeded weights,
five nets covering every activation, 1 / 2 layers, F 32 / 64 / 128, one-hot and sign inputs, reverse order,
y_depth 1..4; gen_gru_yh0_skip: a skip y-MLP)."""
import numpy as np
import pytest
import torch

from conftest import golden

CASES = ["gru_yh0_polar_64_32", "gru_yh0_polar_32_16_f128_relu_rev", "gru_yh0_polar_16_8_l1_tanh_noonehot",
         "gru_yh0_polar_32_16_elu_d1", "gru_yh0_polar_16_8_sigmoid", "gru_yh0_polar_32_16_skip"]


def skip_of(d):
    """gen_gru_yh0_skip: RNN_Model(..., skip=True) -- get_h0 puts y in front of the MLP output (rnn_all.py:369-370)."""
    return bool(int(d["skip"])) if "skip" in d.files else False


def load(name):
    d = golden(f"{name}.npz")
    sd = {k[2:]: d[k] for k in d.files if k.startswith("w.")}
    return d, sd


@pytest.mark.parametrize("name", CASES)
def test_oracle_yh0_matches_reference(oracle, name):
    d, sd = load(name)
    N, F, L = int(d["N"]), int(d["F"]), int(d["layers"])
    act = bytes(d["activation"]).decode()
    y = d["y"]
    x = oracle.ymlp_f64(y, sd, act, int(d["y_depth"]))
    if skip_of(d):
        x = np.concatenate([y.astype(np.float64), x], 1)
    assert np.abs(x - d["h0x"]).max() < 1e-5  # the reference's fp32 MLP against float64
    dec, lg = oracle.gru_decode_f64(y, sd, N, F, L, d["info"], onehot=bool(d["onehot"]), h0x=x, rev=bool(d["rev"]))
    ref = d["decoded"]
    info = d["info"]
    assert (dec[:, info] == ref[:, info]).mean() >= 0.999
    same = (dec[:, info] == ref[:, info]).all(1)
    assert same.mean() >= 0.99
    assert np.abs(lg[same] - d["logits"][same]).max() < 2e-5
    assert np.all(dec[:, np.setdiff1d(np.arange(N), info)] == 1.0)


@pytest.mark.parametrize("name", CASES)
def test_rnn_model_get_h0_matches_reference(name):
    """The package's RNN_Model builds the reference's y_linears (same names and shapes) and get_h0 reproduces the
    reference's initial states, including the activation after the last layer."""
    from neural_polar_decoder_amd.rnn import RNN_Model
    d, sd = load(name)
    N, F, L = int(d["N"]), int(d["F"]), int(d["layers"])
    net = RNN_Model("GRU", 1 + int(d["onehot"]), F, 1, L, N, int(d["y_hidden"]), int(d["y_depth"]),
                    bytes(d["activation"]).decode(), 0.0, skip_of(d))
    net.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    assert net.fused_supported("y_h0") and not net.fused_supported("y_input")
    with torch.no_grad():
        h0 = net.get_h0(torch.from_numpy(d["y"]))
    x = h0.permute(1, 2, 0).reshape(d["y"].shape[0], -1).numpy()
    assert np.abs(x - d["h0x"]).max() < 1e-6


@pytest.mark.parametrize("out_linear_depth", [1, 3])
def test_rnn_from_checkpoint_y_h0(out_linear_depth):
    """A y_h0 checkpoint in the reference's format ({'net': state_dict, 'args': Namespace}, rnn_all.py:1310-1330)
    loads with its y-MLP through datasets.rnn_from_checkpoint and reproduces the reference's initial states.  The
    reference builds y_h0 nets with a one-layer head whatever --out_linear_depth says (rnn_all.py:1317), so a
    checkpoint saved with --out_linear_depth 3 holds 'linear.weight' and must load the same way."""
    import argparse
    from neural_polar_decoder_amd.datasets import rnn_from_checkpoint
    d, sd = load("gru_yh0_polar_64_32")
    args = argparse.Namespace(decoding_type="y_h0", onehot=True, N=64, K=32, rnn_feature_size=64, rnn_depth=2,
                              y_hidden_size=int(d["y_hidden"]), y_depth=int(d["y_depth"]), activation="selu",
                              code="Polar", rate_profile="polar", target_K=32, rnn_type="GRU",
                              out_linear_depth=out_linear_depth)
    net, dec, code = rnn_from_checkpoint({"net": {k: torch.from_numpy(v) for k, v in sd.items()}, "args": args},
                                         device="cpu")
    assert dec.decoding_type == "y_h0" and net.fused_supported("y_h0")
    assert np.array_equal(np.asarray(code.info_positions), d["info"])
    with torch.no_grad():
        h0 = net.get_h0(torch.from_numpy(d["y"]))
    assert np.abs(h0.permute(1, 2, 0).reshape(d["y"].shape[0], -1).numpy() - d["h0x"]).max() < 1e-6
