"""Decode time of the round-4 RNN variants on 2^20 Polar(64,32) words (cuda:0): y_h0 (hidden 64, 2 layers, selu
y-MLP 64 -> 128 -> 128 -> 128) on fp32 and fp16x3 against y_input, and an LSTM (hidden 64, 1 layer) against a GRU of
the same shape.  Seeded PyTorch-default weights.  python tools/rnn_variants_time.py"""
import sys

import torch

sys.path.insert(0, ".")
from neural_polar_decoder_amd import reference_polar_code  # noqa: E402
from neural_polar_decoder_amd.rnn import RNN_decoder, RNN_Model  # noqa: E402

code = reference_polar_code(64, 32)
_, _, y = code.mc_generate(1 << 20, 2.0, 1234, 0, 0, want_msg=False)
info = code.info_positions


def timed(net, dec):
    dec.decode(net, False, y[:4096])
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(3):
        dec.decode(net, False, y)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / 3


torch.manual_seed(1)
rows = []
for kind, cell, L, dtype_in, yh, yd in (("y_input GRU", "GRU", 2, "y_input", 0, 0), ("y_h0 GRU", "GRU", 2, "y_h0", 128, 3),
                                        ("y_input GRU 1 layer", "GRU", 1, "y_input", 0, 0),
                                        ("y_input LSTM 1 layer", "LSTM", 1, "y_input", 0, 0)):
    din = (64 if dtype_in == "y_input" else 0) + 2
    net = RNN_Model(cell, din, 64, 1, L, 64, yh, yd, "selu").cuda().eval()
    precs = ("fp32", "fp16x3") if cell == "GRU" and L == 2 else ("fp32",)
    for prec in precs:
        ms = timed(net, RNN_decoder(dtype_in, 64, info, onehot=True, precision=prec))
        print(f"{kind:22s} {prec:7s} {ms:8.2f} ms per 2^20  {(1 << 20) / ms * 1e3:.3e} cw/s", flush=True)
