"""--bidirectional RNN decoders (rnn_all.py:307, decode rnn_all.py:442 / :523-547) on the CPU: a bidirectional
nn.GRU / nn.LSTM over the one-step sequence is the one-directional cell of hidden 2F with per-gate [forward, reverse]
rows, a block-diagonal W_hh and both directions reading the same layer input (rnn.pack_gru_weights).  The float64 oracle
decodes that packed 2F cell and must reproduce the reference's golden decisions and logits (tests/golden/gen_golden.py
gen_rnn_bi: GRU F 32 x 2 layers, GRU F 64 x 1 layer reversed, LSTM F 16 x 2 layers, y_h0 GRU F 32 x 2 layers) under
the y_input fixtures' bars: >= 99.9 % of information bits and >= 99 % of codewords identical, logits of agreeing
codewords within 2e-5."""
import numpy as np
import pytest
import torch

from conftest import golden

CASES = ["gru_bi_polar_32_16_f32_l2", "gru_bi_polar_16_8_f64_l1_rev", "lstm_bi_polar_16_8_f16_l2",
         "gru_yh0_bi_polar_32_16"]


def build(name):
    """(fixture, this package's RNN_Model holding the reference's bidirectional weights, decoding type)"""
    from neural_polar_decoder_amd.rnn import RNN_Model
    d = golden(f"{name}.npz")
    N, F, L = int(d["N"]), int(d["F"]), int(d["layers"])
    cell, dt = bytes(d["cell"]).decode(), bytes(d["decoding_type"]).decode()
    onehot = bool(d["onehot"])
    din = (N if dt == "y_input" else 0) + 1 + int(onehot)
    yh, yd = (int(d["y_hidden"]), int(d["y_depth"])) if dt == "y_h0" else (0, 0)
    net = RNN_Model(cell, din, F, 1, L, N, yh, yd, "relu", 0.0, False, bidirectional=True)
    net.load_state_dict({k[2:]: torch.from_numpy(d[k]) for k in d.files if k.startswith("w.")})
    return d, net.eval(), dt


def packed_state_dict(net):
    """The packed 2F cell (pack_gru_weights, no y columns) as a one-directional state dict for the oracle."""
    from neural_polar_decoder_amd.rnn import pack_gru_weights
    W = pack_gru_weights(net, net.num_rnn_layers)
    F2, L = 2 * net.feature_size, net.num_rnn_layers
    G = 4 if net.rnn_type == "LSTM" else 3
    sd, off = {}, 0
    for l in range(L):
        din = net.input_size if l == 0 else F2
        for nm, shape in (("weight_ih", (G * F2, din)), ("weight_hh", (G * F2, F2)), ("bias_ih", (G * F2,)),
                          ("bias_hh", (G * F2,))):
            n = int(np.prod(shape))
            sd[f"rnn.{nm}_l{l}"] = W[off:off + n].reshape(shape)
            off += n
    sd["linear.weight"] = W[off:off + F2].reshape(1, F2)
    sd["linear.bias"] = W[off + F2:off + F2 + 1]
    return sd


@pytest.mark.parametrize("name", CASES)
def test_packed_bidirectional_oracle_matches_reference(oracle, name):
    d, net, dt = build(name)
    assert net.fused_supported(dt)
    N, L = int(d["N"]), int(d["layers"])
    F2 = 2 * int(d["F"])
    h0x = None
    if dt == "y_h0":
        x = torch.from_numpy(d["h0x"])
        h0x = x.view(x.shape[0], F2 // 2, L, 2).permute(0, 3, 1, 2).reshape(x.shape[0], -1).numpy()
    dec, lg = oracle.gru_decode_f64(d["y"], packed_state_dict(net), N, F2, L, d["info"], onehot=bool(d["onehot"]),
                                    rev=bool(d["rev"]), h0x=h0x, cell=bytes(d["cell"]).decode())
    info = d["info"]
    ref = d["decoded"]
    assert (dec[:, info] == ref[:, info]).mean() >= 0.999
    same = (dec[:, info] == ref[:, info]).all(1)
    assert same.mean() >= 0.99
    assert np.abs(lg[same] - d["logits"][same]).max() < 2e-5


def test_bidirectional_h0_layout():
    """get_h0's (2 L, B, F) states (index layer 2 + direction) land on the packed cell's unit (dir F + f) of layer l."""
    from neural_polar_decoder_amd.rnn import RNN_Model
    torch.manual_seed(0)
    net = RNN_Model("GRU", 2, 8, 1, 2, 16, 32, 2, "relu", 0.0, False, bidirectional=True).eval()
    y = torch.randn(3, 16)
    with torch.no_grad():
        h = net.get_h0(y)  # (4, 3, 8)
        flat = h.permute(1, 2, 0).reshape(3, -1)  # x layout f 2L + j
    got = flat.view(3, 8, 2, 2).permute(0, 3, 1, 2).reshape(3, -1)  # the decoder's remap
    for l in range(2):
        for dr in range(2):
            for f in range(8):
                assert torch.equal(got[:, (dr * 8 + f) * 2 + l], h[2 * l + dr, :, f])
