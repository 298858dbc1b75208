"""--use_layernorm nets on the MI355X (npd_rnn_create_ex: LayerNorm(F) head on the fp32 GRU kernel, rnn_all.py:317-320,
:387-398) against the reference's golden decisions and logits (tests/golden/gen_golden.py gen_gru_ln), the y_input
bars: >= 99.9 % of information bits and >= 99 % of codewords identical, logits of agreeing codewords within 2e-5; and the
float64 oracle on a ragged batch of fresh words."""
import numpy as np
import pytest
import torch

from conftest import golden

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
CASES = ["gru_ln_polar_32_16", "gru_ln_polar_16_8_l1_noonehot_rev", "gru_ln_yh0_polar_32_16_f32"]


def build(name):
    from neural_polar_decoder_amd.rnn import RNN_decoder, RNN_Model
    d = golden(f"{name}.npz")
    N, F, L = int(d["N"]), int(d["F"]), int(d["layers"])
    dt = bytes(d["decoding_type"]).decode()
    net = RNN_Model("GRU", (N if dt == "y_input" else 0) + 1 + int(d["onehot"]), F, 1, L, N, int(d["y_hidden"]),
                    int(d["y_depth"]), bytes(d["activation"]).decode(), 0.0, False, use_layernorm=True).to(DEV).eval()
    net.load_state_dict({k[2:]: torch.from_numpy(d[k]) for k in d.files if k.startswith("w.")})
    return d, net, RNN_decoder(dt, N, d["info"], onehot=bool(d["onehot"]), reverse_order=bool(d["rev"]))


@pytest.mark.parametrize("name", CASES)
def test_ln_decode_matches_reference(name):
    d, net, dec = build(name)
    info = d["info"]
    out, lg = dec.decode(net, False, torch.from_numpy(d["y"]).to(DEV), return_logits=True)
    out, lg = out.cpu().numpy(), lg.cpu().numpy()
    ref = d["decoded"]
    assert (out[:, info] == ref[:, info]).mean() >= 0.999
    same = (out == ref).all(1)
    assert same.mean() >= 0.99
    assert np.abs(lg[same] - d["logits"][same]).max() < 2e-5


@pytest.mark.parametrize("name", ["gru_ln_polar_32_16", "gru_ln_yh0_polar_32_16_f32"])
def test_ln_decode_vs_oracle_ragged(oracle, name):
    d, net, dec = build(name)
    from neural_polar_decoder_amd import reference_polar_code
    N, F, L = int(d["N"]), int(d["F"]), int(d["layers"])
    code = reference_polar_code(N, int(d["K"]))
    _, _, y = code.mc_generate(3000 + 7, 1.5, seed=9, device=DEV, want_msg=False)
    out, lg = dec.decode(net, False, y, return_logits=True)
    sd = {k[2:]: d[k] for k in d.files if k.startswith("w.")}
    yh = y.cpu().numpy()[::13]
    h0x = None
    if bytes(d["decoding_type"]).decode() == "y_h0":
        h0x = oracle.ymlp_f64(yh, sd, bytes(d["activation"]).decode(), int(d["y_depth"]))
    od, ol = oracle.gru_decode_f64(yh, sd, N, F, L, d["info"], onehot=bool(d["onehot"]), h0x=h0x,
                                   ln_eps=float(d["ln_eps"]))
    o = out.cpu().numpy()[::13]
    same = (o == od).all(1)
    assert same.mean() >= 0.99
    assert np.abs(lg.cpu().numpy()[::13][same] - ol[same]).max() < 2e-5


def test_ln_split_precision_rejected():
    from neural_polar_decoder_amd._lib import NpdError
    from neural_polar_decoder_amd.rnn import RNN_decoder
    d, net, _ = build("gru_ln_polar_32_16")
    dec = RNN_decoder("y_input", int(d["N"]), d["info"], onehot=True, precision="fp16x3")
    with pytest.raises(NpdError):
        dec.decode(net, False, torch.from_numpy(d["y"][:16]).to(DEV))
