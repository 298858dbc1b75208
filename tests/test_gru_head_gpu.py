"""--out_linear_depth > 1 heads on the MI355X (npd_rnn_create_ex: each head layer an fp32 MFMA GEMM per decoding step in
gru_decode_kernel<F, L, 4, HDT>, H padded to 32 HDT) against the reference's golden decisions and logits
(tests/golden/gen_golden.py gen_gru_head), the y_input bars: >= 99.9 % of information bits and >= 99 % of codewords
identical, logits of agreeing codewords within 2e-5; and the float64 oracle on a ragged batch of fresh words."""
import numpy as np
import pytest
import torch

from conftest import golden

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
CASES = ["gru_head_polar_32_16_d2_h64", "gru_head_polar_16_8_d3_h48_noonehot_rev", "gru_head_polar_32_16_f32_d2_h128",
         "gru_head_bi_polar_32_16_f32_d2_h64"]


def build(name):
    from neural_polar_decoder_amd.rnn import RNN_decoder, RNN_Model
    d = golden(f"{name}.npz")
    N, F, L = int(d["N"]), int(d["F"]), int(d["layers"])
    bi = "bidirectional" in d.files and int(d["bidirectional"]) == 1
    net = RNN_Model("GRU", N + 1 + int(d["onehot"]), F, 1, L, N, int(d["y_hidden"]), 0, "selu", 0.0, False,
                    out_linear_depth=int(d["out_linear_depth"]), bidirectional=bi).to(DEV).eval()
    net.load_state_dict({k[2:]: torch.from_numpy(d[k]) for k in d.files if k.startswith("w.")})
    return d, net, RNN_decoder("y_input", N, d["info"], onehot=bool(d["onehot"]), reverse_order=bool(d["rev"]))


@pytest.mark.parametrize("name", CASES)
def test_head_decode_matches_reference(name):
    d, net, dec = build(name)
    info = d["info"]
    out, lg = dec.decode(net, False, torch.from_numpy(d["y"]).to(DEV), return_logits=True)
    out, lg = out.cpu().numpy(), lg.cpu().numpy()
    ref = d["decoded"]
    assert (out[:, info] == ref[:, info]).mean() >= 0.999
    same = (out == ref).all(1)
    assert same.mean() >= 0.99
    assert np.abs(lg[same] - d["logits"][same]).max() < 2e-5


@pytest.mark.parametrize("name", ["gru_head_polar_32_16_d2_h64", "gru_head_polar_32_16_f32_d2_h128"])
def test_head_decode_vs_oracle_ragged(oracle, name):
    d, net, dec = build(name)
    from neural_polar_decoder_amd import reference_polar_code
    N, F, L = int(d["N"]), int(d["F"]), int(d["layers"])
    code = reference_polar_code(N, int(d["K"]))
    _, _, y = code.mc_generate(3000 + 11, 1.5, seed=12, device=DEV, want_msg=False)
    out, lg = dec.decode(net, False, y, return_logits=True)
    sd = {k[2:]: d[k] for k in d.files if k.startswith("w.")}
    yh = y.cpu().numpy()[::13]
    od, ol = oracle.gru_decode_f64(yh, sd, N, F, L, d["info"], onehot=bool(d["onehot"]))
    o = out.cpu().numpy()[::13]
    same = (o == od).all(1)
    assert same.mean() >= 0.99
    assert np.abs(lg.cpu().numpy()[::13][same] - ol[same]).max() < 2e-5
