"""RNN_Model.fused_supported mirrors npd_rnn_create / npd_gru_decode_ex's limits (CPU: no handle is built).

A net the check accepts must not fail later inside handle creation, and a net the kernels cannot run must be
reported unsupported up front (bidirectional hidden 256 x 2 layers at N > 128, packed hidden > 64 in a
split precision)."""
from neural_polar_decoder_amd.rnn import RNN_Model


def gru(F, L, N=64, bi=False, y_hidden=0, y_depth=0, rnn="GRU"):
    return RNN_Model(rnn, (N if y_depth == 0 else 0) + 2, F, 1, L, N, y_hidden, y_depth, bidirectional=bi)


def test_shape_limits_fp32():
    assert gru(512, 2).fused_supported("y_input", "fp32", 128)
    # hidden 512 x 2 layers: both states + the tile's y exceed 160 KB of LDS beyond N = 128
    assert not gru(512, 2, N=256).fused_supported("y_input", "fp32", 256)
    # bidirectional hidden 256 = packed 512: the same bound
    assert gru(256, 2, N=128, bi=True).fused_supported("y_input", "fp32", 128)
    assert not gru(256, 2, N=256, bi=True).fused_supported("y_input", "fp32", 256)
    assert gru(512, 1, N=256).fused_supported("y_input", "fp32", 256)
    assert not gru(64, 2, N=12).fused_supported("y_input", "fp32", 12)
    # without N the check is the shape-only one the callers used before
    assert gru(512, 2, N=256).fused_supported("y_input")


def test_split_precision_limits():
    assert gru(64, 2).fused_supported("y_input", "fp16x3", 64)
    assert gru(32, 1).fused_supported("y_input", "bf16x3", 32)
    assert not gru(128, 2).fused_supported("y_input", "fp16x3", 64)         # split kernels: hidden <= 64
    assert not gru(64, 2, bi=True).fused_supported("y_input", "fp16x3", 64)  # packed 128
    assert gru(32, 2, bi=True).fused_supported("y_input", "fp16x3", 64)      # packed 64
    assert not gru(64, 2, N=24).fused_supported("y_input", "fp16x3", 24)     # N % 16
    # y_h0 in a split precision: the 16-codeword kernel only (hidden 64, 2 layers, N % 32 == 0)
    assert gru(64, 2, y_hidden=128, y_depth=2).fused_supported("y_h0", "fp16x3", 64)
    assert not gru(32, 2, y_hidden=64, y_depth=2).fused_supported("y_h0", "fp16x3", 64)
    assert not gru(64, 2, N=48, y_hidden=128, y_depth=2).fused_supported("y_h0", "fp16x3", 48)
    assert not gru(64, 1, rnn="LSTM").fused_supported("y_input", "fp16x3", 64)  # LSTM cells: fp32 only
