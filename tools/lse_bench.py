"""Exact-LSE SC kernel timing (Polar(64,32) and (256,128), 2 dB, hard/soft) + a parity spot check."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
from neural_polar_decoder_amd import reference_polar_code
from oracle import oracle as O
for N, K, B in [(64, 32, 1 << 18), (128, 64, 1 << 17), (256, 128, 1 << 16)]:
    code = reference_polar_code(N, K)
    _, _, y = code.mc_generate(B, 2.0, 1234, 0, 0, want_msg=False)
    for hard in (False, True):
        h = code.sc_decode(y, 2.0, hard_decision=hard)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(3):
            code.sc_decode(y, 2.0, hard_decision=hard)
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / 3
        oh, _ = O.sc_decode_lse(y[:4096].cpu().numpy(), 2.0, code.info_positions, hard)
        ag = (h[:4096].cpu().numpy() == oh).mean()
        print(f"N={N} hard={hard} {ms:.3f} ms  {B / ms * 1e3:.3e} cw/s  agree={ag:.5f}", flush=True)
