"""--bidirectional RNN decoders on the MI355X: RNN_decoder.decode(net, False, y) runs the packed hidden-2F cell
(rnn.pack_gru_weights; tests/test_rnn_bi.py pins the packing against the reference on the CPU) on the fused kernels --
gru_decode_kernel / gru_wide_kernel / lstm_decode_kernel, and the fp16x3 split kernel where the packed cell is its shape
(2F = 64, 2 layers) -- against the reference's golden decisions and logits (gen_golden.py gen_rnn_bi), the y_input
fixtures' bars."""
import numpy as np
import pytest
import torch

from conftest import golden

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
CASES = ["gru_bi_polar_32_16_f32_l2", "gru_bi_polar_16_8_f64_l1_rev", "lstm_bi_polar_16_8_f16_l2",
         "gru_yh0_bi_polar_32_16"]
SPLIT_OK = {"gru_bi_polar_32_16_f32_l2", "gru_yh0_bi_polar_32_16"}


@pytest.mark.parametrize("precision", ["fp32", "fp16x3"])
@pytest.mark.parametrize("name", CASES)
def test_bidirectional_decode_matches_reference(name, precision):
    from neural_polar_decoder_amd.rnn import RNN_decoder, RNN_Model
    if precision != "fp32" and name not in SPLIT_OK:
        pytest.skip("the split kernel covers the packed 2F = 64, 2-layer GRU")
    d = golden(f"{name}.npz")
    N, F, L = int(d["N"]), int(d["F"]), int(d["layers"])
    cell, dt = bytes(d["cell"]).decode(), bytes(d["decoding_type"]).decode()
    onehot = bool(d["onehot"])
    din = (N if dt == "y_input" else 0) + 1 + int(onehot)
    yh, yd = (int(d["y_hidden"]), int(d["y_depth"])) if dt == "y_h0" else (0, 0)
    net = RNN_Model(cell, din, F, 1, L, N, yh, yd, "relu", 0.0, False, bidirectional=True).to(DEV).eval()
    net.load_state_dict({k[2:]: torch.from_numpy(d[k]) for k in d.files if k.startswith("w.")})
    dec = RNN_decoder(dt, N, d["info"], onehot=onehot, reverse_order=bool(d["rev"]), precision=precision)
    out, lg = dec.decode(net, False, torch.from_numpy(d["y"]).to(DEV), return_logits=True)
    got = out.cpu().numpy()
    info = d["info"]
    assert (got[:, info] == d["decoded"][:, info]).mean() >= 0.999
    same = (got[:, info] == d["decoded"][:, info]).all(1)
    assert same.mean() >= 0.99
    assert np.abs(lg.cpu().numpy()[same] - d["logits"][same]).max() < 2e-5
