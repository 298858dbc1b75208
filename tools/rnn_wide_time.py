"""Decode time of the round-5 RNN additions on Polar(64,32) words (cuda:0, seeded PyTorch-default weights): LSTM cells
on lstm_wide_kernel (hidden 64 x 2 layers, 128 / 256 / 512 x 2 layers) beside GRUs of the same shape, and a
bidirectional GRU (hidden 32 x 2 layers, run as the hidden-64 cell) on fp32 and fp16x3.
python tools/rnn_wide_time.py"""
import sys

import torch

sys.path.insert(0, ".")
from neural_polar_decoder_amd import reference_polar_code  # noqa: E402
from neural_polar_decoder_amd.rnn import RNN_decoder, RNN_Model  # noqa: E402

code = reference_polar_code(64, 32)
info = code.info_positions


def timed(net, dec, y):
    dec.decode(net, False, y[:4096])
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(2):
        dec.decode(net, False, y)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / 2


torch.manual_seed(1)
for F, B in ((64, 1 << 20), (128, 1 << 18), (256, 1 << 16), (512, 1 << 15)):
    _, _, y = code.mc_generate(B, 2.0, 1234, 0, 0, want_msg=False)
    for cell in ("GRU", "LSTM"):
        net = RNN_Model(cell, 66, F, 1, 2, 64, 0, 0).cuda().eval()
        ms = timed(net, RNN_decoder("y_input", 64, info, onehot=True), y)
        print(f"{cell:4s} F {F:3d} x 2 layers fp32    {ms:8.2f} ms per {B:7d}  {B / ms * 1e3:.3e} cw/s", flush=True)
_, _, y = code.mc_generate(1 << 20, 2.0, 1234, 0, 0, want_msg=False)
net = RNN_Model("GRU", 66, 32, 1, 2, 64, 0, 0, bidirectional=True).cuda().eval()
for prec in ("fp32", "fp16x3"):
    ms = timed(net, RNN_decoder("y_input", 64, info, onehot=True, precision=prec), y)
    print(f"GRU bidirectional F 32 x 2 layers {prec:7s} {ms:8.2f} ms per 2^20  {(1 << 20) / ms * 1e3:.3e} cw/s", flush=True)
