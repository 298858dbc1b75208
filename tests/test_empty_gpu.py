"""Empty batches through every decoder surface: no launch, no error, outputs of the reference's shapes with zero
rows, device counters untouched.  Where the reference itself fails on B = 0 the mirror fails the same way:
errors_ber / errors_bler start with y.view(B, -1, 1) (utils.py:20, :38), a RuntimeError for an empty tensor."""
import argparse

import numpy as np
import pytest
import torch

from conftest import trained_fixture

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def test_polar_and_pac_empty():
    from neural_polar_decoder_amd import PAC, reference_polar_code
    code = reference_polar_code(64, 32)
    x = code.encode_plotkin(torch.zeros(0, 32, device=DEV))
    assert x.shape == (0, 64)
    y = code.channel(x, 2.0)
    assert y.shape == (0, 64)
    llr, hat = code.sc_decode_new(y, 2.0)
    assert llr.shape == (0, 64) and hat.shape == (0, 32)
    out = code.scl_decode(y, 2.0, 4)
    assert all(t.shape[0] == 0 for t in (out if isinstance(out, tuple) else (out,)) if torch.is_tensor(t))
    c = torch.zeros(2, dtype=torch.int64, device=DEV)
    code.sc_decode_mc(y, 2.0, 1, 0, c)
    assert int(c.abs().sum()) == 0
    pac = PAC(argparse.Namespace(target_K=64), 128, 64, 91)
    xp = pac.pac_encode(torch.zeros(0, 64, device=DEV))
    assert xp.shape == (0, 128)
    res = pac.pac_sc_decode(pac.channel(xp, 2.0), 2.0)
    assert all(t.shape[0] == 0 for t in res)


def test_counters_on_empty():
    from neural_polar_decoder_amd import errors_ber, errors_bler
    from neural_polar_decoder_amd.utils import count_errors
    t = torch.zeros(0, 16, device=DEV)
    c = count_errors(t, t)
    assert c.tolist() == [0, 0]
    count_errors(t, torch.zeros(0, 64, device=DEV), c, cols=np.arange(16))
    assert c.tolist() == [0, 0]
    # the reference's errors_ber / errors_bler open with y.view(B, -1, 1), which torch refuses for 0 elements
    for f in (errors_ber, errors_bler):
        with pytest.raises(RuntimeError):
            f(t, t)


@pytest.mark.parametrize("precision", ["fp32", "fp16x3"])
def test_gru_empty(precision):
    from neural_polar_decoder_amd.rnn import RNN_Model, RNN_decoder
    d = trained_fixture("trained_crisp_32_16")
    N, F = int(d["N"]), int(d["F"])
    net = RNN_Model("GRU", N + 2, F, 1, int(d["layers"]), N, 0, 0).to(DEV).eval()
    net.load_state_dict({k[2:]: torch.from_numpy(d[k]) for k in d.files if k.startswith("w.")})
    dec = RNN_decoder("y_input", N, d["info"], onehot=True, precision=precision)
    out = dec.decode(net, False, torch.zeros(0, N, device=DEV))
    assert out.shape == (0, N)
    c = torch.zeros(3, 2, dtype=torch.int64, device=DEV)
    dec.decode_count_sweep(net, torch.zeros(3, 0, N, device=DEV), torch.zeros(0, len(d["info"]), device=DEV), c)
    assert int(c.abs().sum()) == 0


@pytest.mark.parametrize("precision", ["fp32", "fp16x3"])
def test_conv_empty(precision):
    from conftest import conv_weights_from_seed
    from neural_polar_decoder_amd.models import convNet
    E, N = 16, 64
    net = convNet(argparse.Namespace(embed_dim=E, max_len=N, N=N, dont_use_bias=False, dropout=0.0),
                  precision=precision)
    net.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in conv_weights_from_seed(E, N, 3).items()})
    lg, dec = net.eval().logits(torch.zeros(0, N, device=DEV))
    assert lg.shape == (0, N) and dec.shape == (0, N)
