"""Empty batches (B = 0) through every public decode/encode method: the reference's methods take any
batch size, including an empty one (torch ops on (0, N) tensors); the drop-in returns correctly shaped
empty results on the input's device and launches nothing (the C ABI returns NPD_OK for B == 0)."""
import argparse

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _empty(*shape):
    return torch.empty(*shape, dtype=torch.float32, device=DEV)


@pytest.mark.parametrize("N,K", [(64, 32), (256, 128)])
def test_polar_methods_on_empty_batch(N, K):
    from neural_polar_decoder_amd.polar import reference_polar_code
    code = reference_polar_code(N, K)
    x = code.encode_plotkin(_empty(0, K))
    assert x.shape == (0, N) and x.is_cuda
    y = code.channel(x, 2.0)
    assert y.shape == (0, N)
    leaf, hat = code.sc_decode_new(y, 2.0)
    assert leaf.shape == (0, N) and hat.shape == (0, K)
    assert code.sc_decode_msg(y, 2.0).shape == (0, K)
    leaf, hat = code.scl_decode(y, 2.0, 4)
    assert leaf.shape == (0, N) and hat.shape == (0, K)
    leaf, hat = code.scl_decode(y.cpu(), 2.0, 4)  # host in -> host out
    assert hat.shape == (0, K) and not hat.is_cuda
    assert code.sc_decode(y, 2.0).shape[0] == 0
    assert code.sc_decode_soft(y, 2.0).shape[0] == 0


def test_pac_methods_on_empty_batch():
    from neural_polar_decoder_amd.pac_code import PAC
    code = PAC(argparse.Namespace(target_K=64), 128, 64, 91, rate_profile="RM")
    x = code.pac_encode(_empty(0, 64))
    assert x.shape == (0, 128)
    llr, v, u = code.pac_sc_decode(code.channel(x, 2.0), 2.0)
    assert llr.shape == (0, 128) and v.shape == (0, 64) and u.shape == (0, 128)


def test_neural_decoders_on_empty_batch():
    from neural_polar_decoder_amd.montecarlo import seeded_conv, seeded_crisp
    from neural_polar_decoder_amd.polar import reference_polar_code
    code = reference_polar_code(64, 32)
    net, dec = seeded_crisp(code, device=DEV)
    out = dec.decode(net, False, _empty(0, 64))
    assert out.shape == (0, 64)
    conv = seeded_conv(64, embed_dim=16, device=DEV)
    lg, d = conv.logits(_empty(0, 64))
    assert lg.shape[0] == 0 and d.shape[0] == 0
