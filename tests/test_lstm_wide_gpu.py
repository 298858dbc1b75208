"""LSTM cells beyond the LDS-resident kernel (lstm_wide_kernel: hidden 64 with 2 layers, hidden 128-512; the weight
images stream from HBM / L2 as gru_wide_kernel's do): RNN_decoder.decode(net, False, y) of seeded nn.LSTM nets
(PyTorch default init, the reference's own RNN_Model modules) against the float64 oracle (oracle.gru_decode_f64,
cell="LSTM", restating nn.LSTM's step and rnn_all.py:523-547) on ragged batches: y_input (one-hot and sign inputs,
reverse order), --use_ynn and y_h0 ((h, c) = get_h0's x, rnn_all.py:370-375).  Bars: >= 97 % of codewords with
identical decisions, logits of those within 5e-5 (the GRU weight-streaming tests' tolerance scaled for the wider
sums).  Parity here is pinned by the oracle, which tests/test_lstm.py and tests/test_lstm_yh0.py hold to the
reference's golden LSTM fixtures."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
ATOL = 5e-5


def _code(N):
    from neural_polar_decoder_amd import reference_polar_code
    return reference_polar_code(N, N // 2)


@pytest.mark.parametrize("N,F,L,onehot,rev,B", [(32, 64, 2, True, True, 83), (64, 128, 1, False, False, 70),
                                                (32, 128, 2, True, False, 97), (32, 256, 2, True, True, 45),
                                                (16, 512, 1, True, False, 33), (16, 512, 2, False, True, 21)])
def test_lstm_wide_y_input_vs_oracle(oracle, N, F, L, onehot, rev, B):
    from neural_polar_decoder_amd.rnn import RNN_decoder, RNN_Model
    code = _code(N)
    torch.manual_seed(N + F + L)
    net = RNN_Model("LSTM", N + 1 + int(onehot), F, 1, L, N, 0, 0).to(DEV).eval()
    assert net.fused_supported("y_input")
    dec = RNN_decoder("y_input", N, code.info_positions, onehot=onehot, reverse_order=rev)
    _, _, y = code.mc_generate(B, 1.0, seed=7, device=DEV, want_msg=False)
    out, lg = dec.decode(net, False, y, return_logits=True)
    sd = {k: v.detach().cpu().numpy() for k, v in net.state_dict().items()}
    od, ol = oracle.gru_decode_f64(y.cpu().numpy(), sd, N, F, L, code.info_positions, onehot=onehot, rev=rev,
                                   cell="LSTM")
    out, lg = out.cpu().numpy(), lg.cpu().numpy()
    info = code.info_positions
    same = (out[:, info] == od[:, info]).all(1)
    assert same.mean() >= 0.97, same.mean()
    assert np.abs(lg[same] - ol[same]).max() < ATOL


def test_lstm_wide_yh0_vs_oracle(oracle):
    """y_h0 at hidden 128, 2 layers: the y-MLP on npd_ymlp_layer, (h, c) of every layer from its output."""
    from neural_polar_decoder_amd.rnn import RNN_decoder, RNN_Model, _ymlp_forward
    N, F, L, B = 32, 128, 2, 61
    code = _code(N)
    torch.manual_seed(3)
    net = RNN_Model("LSTM", 2, F, 1, L, N, 64, 2, "relu", 0.0, False).to(DEV).eval()
    assert net.fused_supported("y_h0")
    dec = RNN_decoder("y_h0", N, code.info_positions, onehot=True)
    _, _, y = code.mc_generate(B, 1.0, seed=11, device=DEV, want_msg=False)
    out, lg = dec.decode(net, False, y, return_logits=True)
    h0x = _ymlp_forward(net, y).cpu().numpy()
    sd = {k: v.detach().cpu().numpy() for k, v in net.state_dict().items()}
    od, ol = oracle.gru_decode_f64(np.zeros((B, N)), sd, N, F, L, code.info_positions, onehot=True, h0x=h0x,
                                   cell="LSTM")
    out, lg = out.cpu().numpy(), lg.cpu().numpy()
    info = code.info_positions
    same = (out[:, info] == od[:, info]).all(1)
    assert same.mean() >= 0.97, same.mean()
    assert np.abs(lg[same] - ol[same]).max() < ATOL


def test_lstm_ynn_vs_oracle(oracle):
    """--use_ynn with LSTM cells (hidden 64, 2 layers on lstm_wide_kernel): Fy = get_Fy(y) replaces y."""
    from neural_polar_decoder_amd.rnn import RNN_decoder, RNN_Model, _ymlp_forward
    N, F, L, B = 32, 64, 2, 57
    code = _code(N)
    torch.manual_seed(5)
    net = RNN_Model("LSTM", N + 2, F, 1, L, N, 48, 2, "tanh", 0.0, False, y_output_size=N).to(DEV).eval()
    assert net.fused_supported("y_input")
    dec = RNN_decoder("y_input", N, code.info_positions, onehot=True)
    _, _, y = code.mc_generate(B, 1.0, seed=13, device=DEV, want_msg=False)
    out, lg = dec.decode(net, False, y, return_logits=True)
    fy = _ymlp_forward(net, y).cpu().numpy()
    sd = {k: v.detach().cpu().numpy() for k, v in net.state_dict().items()}
    od, ol = oracle.gru_decode_f64(fy, sd, N, F, L, code.info_positions, onehot=True, cell="LSTM")
    out, lg = out.cpu().numpy(), lg.cpu().numpy()
    info = code.info_positions
    same = (out[:, info] == od[:, info]).all(1)
    assert same.mean() >= 0.97, same.mean()
    assert np.abs(lg[same] - ol[same]).max() < ATOL
