"""Debug: GPU exact-LSE SC vs the oracle, agreement statistics per case (no asserts)."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
from oracle import oracle as O
from neural_polar_decoder_amd import PolarCode
from neural_polar_decoder_amd.codes import polar_info_positions

for N, K in [(64, 64), (64, 32), (32, 32), (16, 16), (8, 8), (256, 128)]:
    info = polar_info_positions(N, K)
    code = PolarCode(int(np.log2(N)), K, F=np.setdiff1d(np.arange(N), info))
    rng = np.random.default_rng(N * 7 + K)
    for B in (1, 65, 1000):
        y = (rng.standard_normal((B, N)) * 0.8 + (1 - 2 * (rng.random((B, N)) < 0.5))).astype(np.float32)
        for hard in (True, False):
            h, b = code.sc_decode(torch.from_numpy(y).cuda(), 2.5, hard_decision=hard, return_bits=True)
            oh, ob = O.sc_decode_lse(y, 2.5, info, hard)
            h = h.cpu().numpy(); b = b.cpu().numpy()
            ag = h == oh
            line = f"N={N} K={K} B={B} hard={hard} bits={ag.mean():.5f} rows={ag.all(1).mean():.4f}"
            if not ag.all():
                r = int(np.where(~ag.all(1))[0][0])
                i = int(np.where(b[r] != ob[r])[0][0]) if (b[r] != ob[r]).any() else -1
                line += f" first_row={r} first_pos={i} gpu={b[r][max(i,0):max(i,0)+4]} ora={ob[r][max(i,0):max(i,0)+4]}"
                line += f" nan_gpu={np.isnan(b[r]).sum()} nan_ora={np.isnan(ob[r]).sum()}"
            print(line, flush=True)
# scale-free check: tiny LLRs (no overflow anywhere)
info = polar_info_positions(64, 64)
code = PolarCode(6, 64, F=np.array([], dtype=np.int64))
y = np.random.default_rng(1).standard_normal((1000, 64)).astype(np.float32)
for snr in (-10.0, 0.0, 2.5, 6.0):
    h = code.sc_decode(torch.from_numpy(y).cuda(), snr, hard_decision=True).cpu().numpy()
    oh, _ = O.sc_decode_lse(y, snr, info, True)
    print("rate1 snr", snr, (h == oh).mean(), (h == oh).all(1).mean(), flush=True)
